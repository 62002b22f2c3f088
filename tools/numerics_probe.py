"""Per-parameter gradient error of the fused GPU models / blocks against the bf16-mirrored fp32 CPU
reference (tests/bf16_mirror.py).  Prints one JSON line per case with the worst parameters.

    python tools/numerics_probe.py
"""
import copy
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from bf16_mirror import cos, mirror, rel, round_bf16  # noqa: E402


def model_case(name, shape, nc):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    torch.manual_seed(0)
    base = build_model(name, nc)
    ref = mirror(base)
    gpu = copy.deepcopy(base).cuda()
    x = torch.randn(*shape)
    y = torch.randint(0, nc, (shape[0],))
    lr = OF.cross_entropy(ref(round_bf16(x)), y)
    lr.backward()
    lg = OF.cross_entropy(gpu(x.cuda()), y.cuda())
    lg.backward()
    errs = {n: (rel(pg.grad, pr.grad), cos(pg.grad, pr.grad))
            for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters())}
    worst = sorted(errs.items(), key=lambda kv: -kv[1][0])[:5]
    return {"case": f"{name}{tuple(shape)}", "loss_rel": abs(lg.item() - lr.item()) / abs(lr.item()),
            "max_rel": max(e for e, _ in errs.values()), "min_cos": min(c for _, c in errs.values()),
            "median_rel": sorted(e for e, _ in errs.values())[len(errs) // 2],
            "worst": [(n, round(e, 4), round(c, 5)) for n, (e, c) in worst]}


def block_case(kind, inp, planes, stride, x_shape):
    from pytorch_distributed_nn_amd.models.resnet import BasicBlock, Bottleneck
    torch.manual_seed(0)
    blk = (Bottleneck if kind == "bottleneck" else BasicBlock)(inp, planes, stride,
                                                                "downsample" if kind == "bottleneck" else "shortcut")
    ref = mirror(blk)
    gpu = copy.deepcopy(blk).cuda()
    x = torch.randn(*x_shape)
    xr = round_bf16(x).detach().requires_grad_(True)
    yr = ref(xr)
    g = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(g)
    xg = x.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16).requires_grad_(True)
    yg = gpu.forward_nhwc(xg)
    yg.backward(g.permute(0, 2, 3, 1).contiguous().cuda().to(torch.bfloat16))
    errs = {n: (rel(pg.grad, pr.grad), cos(pg.grad, pr.grad))
            for (n, pr), (_, pg) in zip(ref.named_parameters(), gpu.named_parameters())}
    errs["x"] = (rel(xg.grad, xr.grad.permute(0, 2, 3, 1)), cos(xg.grad, xr.grad.permute(0, 2, 3, 1)))
    errs["y"] = (rel(yg, yr.permute(0, 2, 3, 1)), cos(yg, yr.permute(0, 2, 3, 1)))
    worst = sorted(errs.items(), key=lambda kv: -kv[1][0])[:5]
    return {"case": f"{kind}{(inp, planes, stride)}{tuple(x_shape)}", "max_rel": max(e for e, _ in errs.values()),
            "worst": [(n, round(e, 4), round(c, 5)) for n, (e, c) in worst]}


def main():
    for args in [("bottleneck", 256, 64, 1, (8, 256, 16, 16)), ("bottleneck", 256, 128, 2, (8, 256, 16, 16)),
                 ("bottleneck", 64, 64, 1, (8, 64, 16, 16)), ("basic", 64, 64, 1, (8, 64, 16, 16)),
                 ("basic", 64, 128, 2, (8, 64, 16, 16))]:
        print(json.dumps(block_case(*args)), flush=True)
    for args in [("ResNet18", (32, 3, 32, 32), 10), ("ResNet50", (32, 3, 32, 32), 10),
                 ("resnet50", (32, 3, 64, 64), 1000), ("LeNet", (32, 1, 28, 28), 10)]:
        print(json.dumps(model_case(*args)), flush=True)


if __name__ == "__main__":
    main()
