"""Numerics + speed of the ping-pong GEMM engine (csrc/kernels/gemm_pp.h) against an fp32 torch reference
and against torch (hipBLASLt) on the GPT-2 / square shapes.

    python tools/pp_check.py [--perf-only] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).to(BF)


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


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


def check():
    K.set_pp_mode(2)
    bad = 0
    for (M, N, Kd) in [(256, 256, 32), (512, 256, 64), (1000, 520, 96), (300, 264, 64), (2048, 768, 768),
                       (777, 1536, 224), (4096, 2304, 768)]:
        x, w = rnd(M, Kd), rnd(N, Kd)
        ref = x.float() @ w.float().t()
        y = K.gemm_nt(x, w)
        y32 = K.gemm_nt(x, w, out_f32=True)
        wt = w.t().contiguous()
        yn = K.gemm_nn(x, wt)
        bias = torch.randn(N, device="cuda")
        yb = K.gemm_nt(x, w, bias=bias, relu=True)
        refb = torch.relu(ref + bias)
        errs = dict(nt=rel(y, ref), nt32=rel(y32, ref), nn=rel(yn, ref), nt_bias_relu=rel(yb, refb))
        ok = all(v < 1e-2 for v in errs.values()) and rel(y32, ref) < 1e-5
        bad += not ok
        print(f"check M={M} N={N} K={Kd} " + " ".join(f"{k}={v:.2e}" for k, v in errs.items()) +
              (" OK" if ok else " FAIL"), flush=True)
    # every tile width on an odd shape (duplicate-copy instructions, partial tiles)
    M, N, Kd = 1000, 776, 160
    x, w = rnd(M, Kd), rnd(N, Kd)
    ref = x.float() @ w.float().t()
    for bn in (96, 128, 192, 256, 288):
        K.set_pp_bn(bn)
        e = rel(K.gemm_nt(x, w), ref)
        ok = e < 1e-2
        bad += not ok
        print(f"check bn={bn} M={M} N={N} K={Kd} nt={e:.2e}" + (" OK" if ok else " FAIL"), flush=True)
    K.set_pp_bn(0)
    # weight gradient: out += x^T y, split-K slabs
    for (M, N, Kd) in [(2304, 768, 8192), (768, 768, 1024), (520, 264, 96)]:
        x, y = rnd(Kd, M), rnd(Kd, N)
        base = torch.randn(M, N, device="cuda")
        ref = base + x.float().t() @ y.float()
        for sp in (None, 1, 3):
            out = base.clone()
            K.pp_wgrad(x, y, out, splits=sp)
            e = rel(out, ref)
            ok = e < 1e-5
            bad += not ok
            print(f"check wgrad M={M} N={N} K={Kd} splits={sp} err={e:.2e}" + (" OK" if ok else " FAIL"), flush=True)
    K.set_pp_mode(1)
    return bad


SHAPES = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192), ("gpt2_qkv", 8192, 2304, 768),
          ("gpt2_fc", 8192, 3072, 768), ("gpt2_fc2", 8192, 768, 3072), ("gpt2_head", 8192, 50304, 768),
          ("gpt2_proj", 8192, 768, 768), ("gpt2_fc_dgrad", 8192, 768, 3072), ("gpt2_fc2_dgrad", 8192, 3072, 768)]


def perf():
    res = []
    for name, M, N, Kd in SHAPES:
        x, w = rnd(M, Kd), rnd(N, Kd)
        wt = w.t().contiguous()
        fl = 2.0 * M * N * Kd
        r = {"shape": name, "M": M, "N": N, "K": Kd}
        K.set_pp_mode(0)
        r["old_nt"] = fl / timeit(lambda: K.gemm_nt(x, w)) / 1e9
        K.set_pp_mode(2)
        r["pp_nt"] = fl / timeit(lambda: K.gemm_nt(x, w)) / 1e9
        r["pp_nn"] = fl / timeit(lambda: K.gemm_nn(x, wt)) / 1e9
        for bn in (96, 128, 192, 256, 288):
            K.set_pp_bn(bn)
            r[f"pp{bn}"] = fl / timeit(lambda: K.gemm_nt(x, w)) / 1e9
        K.set_pp_bn(0)
        K.set_pp_mode(1)
        r["torch_nt"] = fl / timeit(lambda: x @ w.t()) / 1e9
        r["torch_nn"] = fl / timeit(lambda: x @ wt) / 1e9
        print(" ".join(f"{k}={v:.0f}" if isinstance(v, float) else f"{k}={v}" for k, v in r.items()), flush=True)
        res.append(r)
    for name, M, N, Kd in [("wg_qkv", 2304, 768, 8192), ("wg_fc", 3072, 768, 8192), ("wg_fc2", 768, 3072, 8192),
                           ("wg_proj", 768, 768, 8192), ("wg_head", 50304, 768, 8192)]:
        x, y = rnd(Kd, M), rnd(Kd, N)
        out = torch.zeros(M, N, device="cuda")
        fl = 2.0 * M * N * Kd
        r = {"shape": name, "M": M, "N": N, "K": Kd}
        r["old_tn"] = fl / timeit(lambda: K.gemm_tn_acc(x, y, out)) / 1e9
        for sp in (None, 1, 2, 4, 8):
            r[f"pp_s{sp}"] = fl / timeit(lambda: K.pp_wgrad(x, y, out, splits=sp)) / 1e9
        r["torch_tn"] = fl / timeit(lambda: torch.addmm(out, x.t(), y, out_dtype=torch.float32, out=out)) / 1e9
        print(" ".join(f"{k}={v:.0f}" if isinstance(v, float) else f"{k}={v}" for k, v in r.items()), flush=True)
        res.append(r)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--perf-only", action="store_true")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    bad = 0 if a.perf_only else check()
    res = perf()
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
