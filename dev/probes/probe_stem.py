"""Time the ImageNet stem kernels at bs256 (stem conv NCHW / NHWC, fused BN+ReLU+max-pool, NCHW->NHWC copy).

python tools/probe_stem.py [--iters N]     (also the program profiled by the stem PMC passes)"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K   # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters * 1e3, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    x = torch.randn(a.batch, 3, 224, 224, device="cuda").to(torch.bfloat16)
    w = torch.randn(64, 3, 7, 7, device="cuda") * 0.1
    w32 = K.stem_weight_nchw(w)
    xin = K.nchw_to_nhwc(x, 8)
    kpad = torch.nn.functional.pad(w.to(torch.bfloat16).permute(0, 2, 3, 1), (0, 5)).contiguous()
    t, _ = K.stem_conv_nchw(x, w32)
    sc, sh = torch.rand(64, device="cuda"), torch.randn(64, device="cuda")
    row = {
        "stem_nchw": timeit(lambda: K.stem_conv_nchw(x, w32), a.iters),
        "stem_nchw_nostats": timeit(lambda: K.stem_conv_nchw(x, w32, want_stats=False), a.iters),
        "stem_nhwc": timeit(lambda: K.stem_conv(xin, kpad), a.iters),
        "nchw_to_nhwc": timeit(lambda: K.nchw_to_nhwc(x, 8), a.iters),
        "bn_relu_maxpool": timeit(lambda: K.bn_relu_maxpool(t, sc, sh), a.iters),
        "generic_conv": timeit(lambda: K.conv_fwd(xin, kpad, 2, 3, want_stats=True), a.iters),
    }
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
