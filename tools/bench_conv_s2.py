"""A/B of ResNet-50's stride-2 3x3 convs (ImageNet, bs 256; the stage-transition Bottlenecks' conv2): the
half-resolution halo kernels (csrc/kernels/conv_s2.hip) vs the implicit-GEMM engine (tuning s2_halo = 0), for the
forward with fused BN statistics (on a materialised a1, and on t1 with the BN + ReLU prologue) and the data gradient
with the fused BN-backward epilogue and the BN2-backward operand prologue -- what the fused Bottleneck runs.

    python tools/bench_conv_s2.py [--batch 256] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd import tuning   # noqa: E402
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402

SHAPES = [(56, 56, 128), (28, 28, 256), (14, 14, 512)]   # input H, W, C (= Ko)


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
    for H, W, C in SHAPES:
        Ho, Wo = H // 2, W // 2
        x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(C, 3, 3, C, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(N, Ho, Wo, C, device="cuda").to(torch.bfloat16)
        t2 = torch.randn(N, Ho, Wo, C, device="cuda").to(torch.bfloat16)
        one, zero = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        g = torch.rand(C, device="cuda") + 0.5
        bn = (x, zero, one, one, zero)
        pre = (t2, zero, one, g, zero, zero, torch.empty_like(dy))
        flops = 2.0 * N * Ho * Wo * C * C * 9
        row = {"shape": [H, W, C]}
        for name, mode in (("gemm", 0), ("halo", 1 | 2 | 8 | 16 | 32)):
            old = tuning.set("s2_halo", mode)
            r = {"fwd_us": timeit(lambda: K.conv_fwd(x, w, 2, 1, want_stats=True), a.iters)}
            if mode:
                r["fwd_pro_us"] = timeit(lambda: K.conv_fwd(x, w, 2, 1, want_stats=True, pro=(one, zero)), a.iters)
                r["dgrad_pre_us"] = timeit(lambda: K.conv_dgrad(dy, w, x.shape, 2, 1, bn=bn, pre=pre), a.iters)
            r["dgrad_us"] = timeit(lambda: K.conv_dgrad(dy, w, x.shape, 2, 1, bn=bn), a.iters)
            if mode:
                tuning.set("s2_halo", mode | 128)
                r["dgrad_pair_us"] = timeit(lambda: K.conv_dgrad(dy, w, x.shape, 2, 1, bn=bn), a.iters)
                tuning.set("s2_halo", mode)
                a1 = torch.empty_like(x)
                r["fwd_pro_a1_us"] = timeit(lambda: K.conv3x3s2(x, w, want_stats=True, pro=(one, zero), pro_out=a1),
                                            a.iters)
            dw = torch.zeros(C, 3, 3, C, device="cuda")
            r["wgrad_us"] = timeit(lambda: K.conv_wgrad(x, dy, 3, 3, 2, 1, out=dw), a.iters)
            r["wgrad_pro_us"] = timeit(lambda: K.conv_wgrad(x, dy, 3, 3, 2, 1, pro=(one, zero), out=dw), a.iters)
            tuning.set("s2_halo", old)
            for k in list(r):
                r[k] = round(r[k], 1)
                r[k.replace("_us", "_tflops")] = round(flops / r[k] / 1e6, 1)
            row[name] = r
            tot[name] = tot.get(name, 0.0) + r["fwd_us"] + r["dgrad_us"] + r["wgrad_us"]
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_fwd_dgrad_wgrad_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
