"""GEMM engine microbenchmark vs torch (hipBLASLt) on the shapes of the flagship models.

    python tools/bench_gemm.py [--zero]      # prints TF/s per shape for ours and torch
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

SHAPES = [  # (name, M, N, K)
    ("sq4096", 4096, 4096, 4096),
    ("sq8192", 8192, 8192, 8192),
    ("gpt2_qkv", 8192, 2304, 768),
    ("gpt2_fc", 8192, 3072, 768),
    ("gpt2_fc2", 8192, 768, 3072),
    ("gpt2_head", 8192, 50304, 768),
    ("r50_1x1_256_64", 802816, 64, 256),
    ("r50_1x1_64_256", 802816, 256, 64),
    ("r50_1x1_1024_256", 50176, 256, 1024),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--zero", action="store_true")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    res = []
    for name, M, N, Kd in SHAPES:
        mk = torch.zeros if a.zero else torch.randn
        x = mk(M, Kd, device="cuda").to(torch.bfloat16)
        w = mk(N, Kd, device="cuda").to(torch.bfloat16)
        wt = w.t().contiguous()
        g = mk(M, N, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(N, Kd, device="cuda")
        fl = 2.0 * M * N * Kd
        r = {"shape": name, "M": M, "N": N, "K": Kd}
        r["ours_nt"] = fl / timeit(lambda: K.gemm_nt(x, w)) / 1e9
        r["torch_nt"] = fl / timeit(lambda: x @ w.t()) / 1e9
        r["ours_nn"] = fl / timeit(lambda: K.gemm_nn(x, wt)) / 1e9
        r["torch_nn"] = fl / timeit(lambda: x @ wt) / 1e9
        r["ours_tn"] = fl / timeit(lambda: K.gemm_tn_acc(g, x, dw)) / 1e9
        r["torch_tn"] = fl / timeit(lambda: g.t() @ x) / 1e9
        if Kd % 128 == 0:
            xq = x.to(torch.float8_e4m3fn).view(torch.uint8)
            wq = w.to(torch.float8_e4m3fn).view(torch.uint8)
            one = torch.ones(1, device="cuda")
            r["ours_fp8_nt"] = fl / timeit(lambda: K.gemm_fp8(xq, wq, one)) / 1e9
        print(" ".join(f"{k}={v:.0f}" if isinstance(v, float) else f"{k}={v}" for k, v in r.items()), flush=True)
        res.append(r)
        del x, w, wt, g, dw
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
