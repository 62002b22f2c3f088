"""Split-count sweeps on the ping-pong engine: the tied LM head's data gradient (gemm_nt_splitk, 8192 x 768 x
50304) and the GPT-2 weight gradients (pp_wgrad, M x N x 8192 tokens) per tile width, against the planned choice.

    python dev/probes/splitk_sweep.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402
from pytorch_distributed_nn_amd.ops._backend import lib  # noqa: E402

BF = torch.bfloat16


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def r(*s, sc=1.0):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * sc).to(BF)


def main():
    M, N, Kd = 8192, 768, 50304
    g, wt = r(M, Kd, sc=0.01), r(N, Kd, sc=0.05)
    ref = K.gemm_nt_splitk(g, wt, splits=1).float()
    out = {"gemm": "head_dgrad", "planned": int(lib().pdnn_pp_splitk_splits(M, N, Kd))}
    for s in (2, 3, 4, 5, 6, 8, 10, 12):
        y = K.gemm_nt_splitk(g, wt, splits=s)
        assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
        out[f"s{s}"] = timeit(lambda: K.gemm_nt_splitk(g, wt, splits=s))
    out["auto"] = timeit(lambda: K.gemm_nt_splitk(g, wt))
    print(json.dumps(out), flush=True)
    T = 8192
    for name, (Mo, No) in {"qkv": (2304, 768), "proj": (768, 768), "fc": (3072, 768), "fc2": (768, 3072)}.items():
        x, y = r(T, Mo), r(T, No)
        o = torch.zeros(Mo, No, device="cuda")
        plan = int(lib().pdnn_pp_wgrad_plan(Mo, No, T, 0))
        res = {"gemm": name + "_wgrad", "plan": plan, "auto": timeit(lambda: K.pp_wgrad(x, y, o))}
        for bn in (128, 256):
            old = K.tune_set("pp_bn", bn)
            for s in (1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 14):
                res[f"bn{bn}_s{s}"] = timeit(lambda: K.pp_wgrad(x, y, o, splits=s))
            K.tune_set("pp_bn", old)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
