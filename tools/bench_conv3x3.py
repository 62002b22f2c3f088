"""A/B of the 3x3 / stride-1 convs of ResNet-50 (ImageNet, bs256): LDS-halo kernel (conv3x3.hip, output
tiles of 64 / 128 channels) vs the implicit-GEMM engine, for the forward with fused BN statistics and the
data gradient with the fused BN-backward epilogue (what the fused bottleneck runs).

    python tools/bench_conv3x3.py [--batch 256] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402

SHAPES = [(56, 56, 64, 3), (28, 28, 128, 4), (14, 14, 256, 6), (7, 7, 512, 3)]   # H, W, C (= Ko), count


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3      # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N = a.batch
    tot = {}
    for H, W, C, cnt in SHAPES:
        x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
        t = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
        mean, inv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        sc, sh = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        flops = 2.0 * N * H * W * C * C * 9
        row = {"shape": [H, W, C], "count": cnt}
        for name, mode, nb in (("gemm", 0, 0), ("halo64", 1, 64), ("halo128", 1, 128), ("w64_resident", 1, 1),
                               ("halo", 1, 0)):
            if (nb == 128 and C % 128) or (nb == 1 and C != 64):
                continue
            old = K.set_conv3x3_mode(mode, nb)
            tf = timeit(lambda: K.conv_fwd(x, w, 1, 1, want_stats=True), a.iters)
            td = timeit(lambda: K.conv_dgrad(x, w, x.shape, 1, 1, bn=(t, mean, inv, sc, sh)), a.iters)
            K.set_conv3x3_mode(*old)
            row[name] = {"fwd_us": round(tf, 1), "dgrad_us": round(td, 1),
                         "fwd_tflops": round(flops / tf / 1e6, 1), "dgrad_tflops": round(flops / td / 1e6, 1)}
            tot.setdefault(name, 0.0)
            tot[name] += cnt * (tf + td)
        print(json.dumps(row), flush=True)
    print(json.dumps({"step_total_us_fwd+dgrad": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
