"""Per-layer benchmark of the HIP implicit-GEMM conv kernels against MIOpen (torch bf16 channels_last)
on every distinct ResNet-50 (ImageNet, 224x224) conv shape, forward / dgrad / wgrad.

    python tools/bench_conv.py --batch 256 [--only fwd] [--json out.json]
"""
import argparse
import json
import time

import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K

# (H, W, C, Ko, R, stride, pad, count-in-resnet50)
SHAPES = [
    (224, 224, 8, 64, 7, 2, 3, 1),
    (56, 56, 64, 64, 1, 1, 0, 1), (56, 56, 64, 64, 3, 1, 1, 3), (56, 56, 64, 256, 1, 1, 0, 4),
    (56, 56, 256, 64, 1, 1, 0, 2),
    (56, 56, 256, 128, 1, 1, 0, 1), (56, 56, 128, 128, 3, 2, 1, 1), (28, 28, 128, 512, 1, 1, 0, 4),
    (56, 56, 256, 512, 1, 2, 0, 1), (28, 28, 512, 128, 1, 1, 0, 3), (28, 28, 128, 128, 3, 1, 1, 3),
    (28, 28, 512, 256, 1, 1, 0, 1), (28, 28, 256, 256, 3, 2, 1, 1), (14, 14, 256, 1024, 1, 1, 0, 6),
    (28, 28, 512, 1024, 1, 2, 0, 1), (14, 14, 1024, 256, 1, 1, 0, 5), (14, 14, 256, 256, 3, 1, 1, 5),
    (14, 14, 1024, 512, 1, 1, 0, 1), (14, 14, 512, 512, 3, 2, 1, 1), (7, 7, 512, 2048, 1, 1, 0, 3),
    (14, 14, 1024, 2048, 1, 2, 0, 1), (7, 7, 2048, 512, 1, 1, 0, 2), (7, 7, 512, 512, 3, 1, 1, 2),
]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--layers", default=None, help="comma-separated indices into SHAPES")
    ap.add_argument("--only", default=None, choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    N = a.batch
    res = []
    tot = {"ours": [0.0, 0.0, 0.0], "miopen": [0.0, 0.0, 0.0]}
    sel = [int(i) for i in a.layers.split(",")] if a.layers else range(len(SHAPES))
    for li in sel:
        (H, W, C, Ko, R, st, pad, cnt) = SHAPES[li]
        x = torch.randn(N, H, W, C, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Ko, R, R, C, device="cuda") * 0.05).to(torch.bfloat16)
        Ho, Wo = K.conv_out_hw(H, W, R, R, st, pad)
        dy = torch.randn(N, Ho, Wo, Ko, device="cuda").to(torch.bfloat16)
        flops = 2.0 * N * Ho * Wo * Ko * C * R * R
        on = lambda k: a.only in (None, k)
        it = a.iters
        t_f = timeit(lambda: K.conv_fwd(x, w, st, pad, want_stats=True), it) if on("fwd") else 1e-9
        t_d = timeit(lambda: K.conv_dgrad(dy, w, x.shape, st, pad), it) if not (R == 7) and on("dgrad") else 1e-9
        t_w = timeit(lambda: K.conv_wgrad(x, dy, R, R, st, pad), it) if on("wgrad") else 1e-9
        row = {"shape": [H, W, C, Ko, R, st, pad], "count": cnt, "ours_ms": [t_f, t_d, t_w],
               "ours_tflops": [flops / t_f / 1e9, flops / max(t_d, 1e-9) / 1e9, flops / t_w / 1e9]}
        for i, t in enumerate((t_f, t_d, t_w)):
            tot["ours"][i] += cnt * t
        if not a.no_ref:
            xc = x.permute(0, 3, 1, 2)  # channels_last NCHW view
            wc = w.permute(0, 3, 1, 2)
            dyc = dy.permute(0, 3, 1, 2)
            r_f = timeit(lambda: F.conv2d(xc, wc, None, st, pad))
            r_b = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [st, st], [pad, pad], [1, 1],
                                                                     False, [0, 0], 1, [R != 7, False, False]))
            r_w = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, [st, st], [pad, pad], [1, 1],
                                                                     False, [0, 0], 1, [False, True, False]))
            row["miopen_ms"] = [r_f, r_b, r_w]
            for i, t in enumerate((r_f, r_b, r_w)):
                tot["miopen"][i] += cnt * t
        res.append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_ms_per_step_fwd_dgrad_wgrad": tot}), flush=True)
    if a.json:
        json.dump({"layers": res, "total": tot}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
