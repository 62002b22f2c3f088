"""Find the first kernel call whose output differs between two identical fused ResNet-50 copies (same weights, buffers,
input) at a step where their gradients differ (dev/probes/det_probe.py): every ops.kernels call is wrapped to record a
float64 fingerprint of each tensor it returns (and of its in-place 'out' / 'acc' / 'pre' outputs)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from pytorch_distributed_nn_amd import tuning  # noqa: E402
from pytorch_distributed_nn_amd.models import build_model  # noqa: E402
from pytorch_distributed_nn_amd.ops import functional as OF  # noqa: E402
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from pytorch_distributed_nn_amd.optim.flat import flatten_module  # noqa: E402

LOG = []
NAMES = ["conv_fwd", "conv_dgrad", "conv_wgrad", "conv3x3", "conv3x3s2", "conv1x1_panel", "bn_apply", "bn_bwd_reduce",
         "bn_bwd_apply", "bn_bwd_finalize", "bn_finalize", "subsample", "conv3x3_flip", "transpose_bf16",
         "stem_conv_nchw", "bn_relu_maxpool", "maxpool_bwd_bnred", "stem_wgrad_nchw"]


def fp(t):
    if isinstance(t, torch.Tensor) and t.is_cuda and t.is_floating_point():
        x = t.detach().double()
        return (tuple(t.shape), round(x.sum().item(), 6), round(x.abs().sum().item(), 6))
    return None


def wrap(name, fn):
    def w(*a, **k):
        r = fn(*a, **k)
        torch.cuda.synchronize()
        outs = r if isinstance(r, tuple) else (r,)
        rec = [fp(o) for o in outs]
        for key in ("out", "acc"):
            v = k.get(key)
            if isinstance(v, (list, tuple)):
                rec += [fp(x) for x in v]
            else:
                rec.append(fp(v))
        pre = k.get("pre")
        if pre is not None and pre[-1] is not None:
            rec.append(("pre_out", fp(pre[-1])))
        LOG.append((name, rec))
        return r
    return w


for n in NAMES:
    if hasattr(K, n):
        setattr(K, n, wrap(n, getattr(K, n)))


def main(step_fail=2, hw=64, bs=4):
    tuning.set("s2_halo", 1)
    tuning.set("ds_sub", 0)
    tuning.set("side_wgrad", 0)
    torch.manual_seed(0)
    dev = torch.device("cuda")
    a = build_model("resnet50").to(dev)
    b = copy.deepcopy(a)
    fa, fb = flatten_module(a), flatten_module(b)
    g = torch.Generator().manual_seed(1)
    for s in range(step_fail + 1):
        fb.data.copy_(fa.data)
        fb.refresh_shadow()
        fa.refresh_shadow()
        for x1, x2 in zip(b.buffers(), a.buffers()):
            x1.copy_(x2)
        x, y = torch.randn(bs, 3, hw, hw, generator=g).to(dev), torch.randint(0, 1000, (bs,), generator=g).to(dev)
        logs = []
        for m, f in ((a, fa), (b, fb)):
            LOG.clear()
            f.zero_grad()
            OF.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            logs.append(list(LOG))
        tot = ((fa.grad - fb.grad).norm() / fb.grad.norm()).item()
        print("step", s, "grad rel diff", tot, "calls", len(logs[0]), len(logs[1]), flush=True)
        if tot > 0:
            for i, (ra, rb) in enumerate(zip(*logs)):
                if ra != rb:
                    print("first differing call", i, ra[0])
                    print("  a:", ra[1])
                    print("  b:", rb[1])
                    for j in range(max(0, i - 3), i):
                        print("  prev", j, logs[0][j][0], logs[0][j][1])
                    break


if __name__ == "__main__":
    main()
