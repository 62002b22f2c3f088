"""Per-tensor first-step gradient agreement of ResNet-50 variants with stock fp32 torch (is a low cosine a
fused-path bug or the fp32 reference's own sensitivity?).

python dev/probes/grad_cos.py [--batch 64 --size 112]
Rows: fused bf16 path; stock torch in bf16; stock fp32 on a 1e-3-perturbed input; fused with each router off."""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def grads(m):
    return [p.grad.detach().float().flatten().clone() for p in m.parameters()]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=112)
    ap.add_argument("--bn3", type=float, default=1.0, help="initial gamma of every residual branch's last BN")
    a = ap.parse_args()
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF, kernels as K
    from pytorch_distributed_nn_amd.optim import flatten_module
    from pytorch_distributed_nn_amd import tuning
    torch.manual_seed(0)
    ref = build_model("resnet50").cuda()
    ref.fused = False
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if n.endswith("bn3.weight"):
                p.fill_(a.bn3)
    names = [n for n, _ in ref.named_parameters()]
    g = torch.Generator().manual_seed(0)
    x = torch.randn(a.batch, 3, a.size, a.size, generator=g).cuda()
    y = torch.randint(0, 1000, (a.batch,), generator=g).cuda()

    def stock(m, xx):
        m.zero_grad()
        torch.nn.functional.cross_entropy(m(xx).float(), y).backward()
        return grads(m)

    base = stock(ref, x)
    rows = {}
    rows["stock fp32, input*(1+1e-3 noise)"] = stock(ref, x * (1 + 1e-3 * torch.randn_like(x)))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        rows["stock torch autocast bf16"] = stock(ref, x)
    rb = copy.deepcopy(ref).to(torch.bfloat16)
    rows["stock torch bf16"] = stock(rb, x.to(torch.bfloat16))
    del rb

    def fused_run(setup=None, undo=None):
        fm = copy.deepcopy(ref)
        fm.fused = True
        fp = flatten_module(fm)
        if setup:
            setup()
        try:
            fp.zero_grad()
            OF.cross_entropy(fm(x.to(torch.bfloat16)), y).backward()
            torch.cuda.synchronize()
        finally:
            if undo:
                undo()
        return grads(fm)

    rows["fused"] = fused_run()
    rows["fused stem mode 0"] = fused_run(lambda: K.set_stem_mode(0), lambda: K.set_stem_mode(2))
    rows["fused conv3x3 off"] = fused_run(lambda: K.set_conv3x3_mode(0), lambda: K.set_conv3x3_mode(1))
    rows["fused panel off"] = fused_run(lambda: K.set_panel_mode(0), lambda: K.set_panel_mode(1))
    rows["fused side_wgrad 0"] = fused_run(lambda: tuning.set("side_wgrad", 0), lambda: tuning.set("side_wgrad", 1))
    groups = ["conv1", "bn1", "layer1.0", "layer1.2", "layer2.0", "layer2.3", "layer3.0", "layer3.5", "layer4.0",
              "layer4.2", "fc"]
    print(f"bn3 gamma {a.bn3}, batch {a.batch}, {a.size}x{a.size}")
    print(f"{'variant':36s} " + " ".join(f"{gname[:9]:>9s}" for gname in groups))
    for k, gs in rows.items():
        cells = []
        for gname in groups:
            cs = [torch.nn.functional.cosine_similarity(gs[i], base[i], dim=0).item()
                  for i, n in enumerate(names) if n == gname + ".weight" or n.startswith(gname + ".")]
            cells.append(min(cs) if cs else float("nan"))
        print(f"{k:36s} " + " ".join(f"{c:9.4f}" for c in cells), flush=True)


if __name__ == "__main__":
    main()
