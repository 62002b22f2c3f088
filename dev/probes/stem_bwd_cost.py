"""The ResNet-50 stem's backward tail in isolation (bs 256): the stem weight gradient (stem_wgrad_nchw, with the stem
BN-backward apply in its staging) warm (back to back) and after a 1 GB write that evicts the caches, and the
max-pool backward with the BN-backward reduce; us per call."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16


def ev_time(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3


def main():
    N = 256
    x = torch.randn(N, 3, 224, 224, device="cuda").to(BF)
    dt = (torch.randn(N, 112, 112, 64, device="cuda") * 0.1).to(BF)
    t = torch.randn(N, 112, 112, 64, device="cuda").to(BF)
    v = [torch.rand(64, device="cuda") + 0.5 for _ in range(8)]
    pre = (t, v[0], v[1], v[2], v[3], v[4], v[5], v[6])
    junk = torch.empty(1 << 28, device="cuda")        # 1 GB
    acc = torch.zeros(64, 3, 7, 7, device="cuda").to(memory_format=torch.channels_last)
    fn = lambda: K.stem_wgrad_nchw(x, dt, pre=pre, acc=acc)   # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    warm = sorted(ev_time(fn) for _ in range(10))
    cold = []
    for _ in range(10):
        junk.fill_(1.0)
        torch.cuda.synchronize()
        cold.append(ev_time(fn))
    out = {"stem_wgrad_warm_us": [round(w, 1) for w in warm], "stem_wgrad_cold_us": sorted(round(c, 1) for c in cold)}
    fn2 = lambda: K.stem_wgrad_nchw(x, dt, acc=acc)   # noqa: E731
    out["stem_wgrad_nopre_warm_us"] = sorted(round(ev_time(fn2), 1) for _ in range(10))
    dy = (torch.randn(N, 56, 56, 64, device="cuda") * 0.1).to(BF)
    idx = torch.randint(0, 9, (N, 56, 56, 64), device="cuda", dtype=torch.uint8)
    fn3 = lambda: K.maxpool_bwd_bnred(dy, idx, t, v[0], v[1], v[2], v[3])   # noqa: E731
    fn3()
    torch.cuda.synchronize()
    out["maxpool_bwd_bnred_us"] = sorted(round(ev_time(fn3), 1) for _ in range(10))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
