"""Loss curve of the tests/test_fp8_gpu.py memorisation run (ResNet-50, 16 images 64x64, 12 SGD steps), bf16 and fp8."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(fp8, seed=0):
    from pytorch_distributed_nn_amd.models import build_model
    from pytorch_distributed_nn_amd.ops import functional as OF
    from pytorch_distributed_nn_amd.optim import SGD, flatten_module
    torch.manual_seed(seed)
    m = build_model("resnet50").cuda()
    if fp8:
        m.enable_fp8()
    flatten_module(m)
    opt = SGD(m.parameters(), lr=0.01, momentum=0.9)
    xin = torch.randn(16, 3, 64, 64, device="cuda")
    yl = torch.randint(0, 10, (16,), device="cuda")
    out = []
    for _ in range(12):
        opt.zero_grad()
        loss = OF.cross_entropy(m(xin), yl)
        loss.backward()
        opt.step()
        out.append(round(loss.item(), 3))
    return out


if __name__ == "__main__":
    for fp8 in (False, True):
        for seed in (0, 1):
            print(json.dumps({"fp8": fp8, "seed": seed, "loss": run(fp8, seed)}), flush=True)
