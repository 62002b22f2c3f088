"""Every GEMM of a GPT-2 small step as the model calls it (fused epilogues included), us per call on the
in-tree ping-pong engine at each tile width, against torch (hipBLASLt, plain / addmm with bias)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16


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
    return round(s.elapsed_time(e) / iters * 1e3, 1)


def r(*s, sc=1.0):
    return ((torch.rand(*s, device="cuda") * 2 - 1) * sc).to(BF)


def main():
    M, D = 8192, 768
    only = sys.argv[1:]
    cases = {
        "qkv_fwd": (D, 3 * D, dict(bias=True)),
        "proj_fwd": (D, D, dict(bias=True, res=True)),
        "fc_fwd": (D, 4 * D, dict(bias=True, act=2)),
        "fc2_fwd": (4 * D, D, dict(bias=True, res=True)),
        "fc2_dgrad": (D, 4 * D, dict(dgelu=True)),
        "fc_dgrad": (4 * D, D, {}),
        "proj_dgrad": (D, D, {}),
        "qkv_dgrad": (3 * D, D, {}),
        "head_fwd": (D, 50304, {}),
    }
    for name, (Kd, N, ep) in cases.items():
        if only and name not in only:
            continue
        x, w = r(M, Kd), r(N, Kd, sc=0.05)
        bias = torch.randn(N, device="cuda") if ep.get("bias") else None
        res = r(M, N) if ep.get("res") else None
        aux = torch.empty(M, N, device="cuda", dtype=BF) if ep.get("act") else None
        dg = r(M, N) if ep.get("dgelu") else None
        fn = lambda: K.gemm_nt_ex(x, w, bias=bias, act=ep.get("act", 0), aux=aux, res=res, dgelu=dg)   # noqa: E731
        out = {"gemm": name, "M": M, "N": N, "K": Kd, "auto": timeit(fn)}
        for bn in (96, 128, 192, 256, 288):
            old = K.tune_set("pp_bn", bn)
            out[f"bn{bn}"] = timeit(fn)
            K.tune_set("pp_bn", old)
        old = K.tune_set("pp_sk64", 0)
        out["auto_sk32"] = timeit(fn)
        for bn in (96, 128):
            ob = K.tune_set("pp_bn", bn)
            out[f"bn{bn}_sk32"] = timeit(fn)
            K.tune_set("pp_bn", ob)
        K.tune_set("pp_sk64", old)
        out["torch"] = timeit(lambda: x @ w.t())
        if bias is not None:
            out["torch_addmm"] = timeit(lambda: torch.addmm(bias.to(BF), x, w.t()))
        out["auto_tflops"] = round(2 * M * N * Kd / out["auto"] / 1e6, 1)
        out["torch_tflops"] = round(2 * M * N * Kd / out["torch"] / 1e6, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
