"""Runs the halo / panel conv kernels at one ResNet-50 shape a few times (PMC / trace target).

    python tools/c3_probe.py --H 56 --C 64 [--kind fwd|dgrad|panel] [--iters 5]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--H", type=int, default=56)
    ap.add_argument("--C", type=int, default=64)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--kind", default="fwd")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    H, C = a.H, a.C
    x = torch.randn(a.N, H, H, C, device="cuda").to(torch.bfloat16)
    t = torch.randn(a.N, H, H, C, device="cuda").to(torch.bfloat16)
    w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
    w1 = (torch.randn(4 * C, 1, 1, C, device="cuda") * 0.05).to(torch.bfloat16)
    mean, inv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    for _ in range(a.iters):
        if a.kind == "fwd":
            K.conv_fwd(x, w, 1, 1, want_stats=True)
        elif a.kind == "dgrad":
            K.conv_dgrad(x, w, x.shape, 1, 1, bn=(t, mean, inv, inv, mean))
        else:
            K.conv_fwd(x, w1, 1, 0, want_stats=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
