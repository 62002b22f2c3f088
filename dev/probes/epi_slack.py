"""A/B of the ping-pong engine's deferred epilogue-store drain (tuning pp_epi_slack) and epilogue pairing
(pp_epi_pair) on every GPT-2 small GEMM
as the model calls it (fused epilogues), us per call; also checks that both settings give the same bits.

    python dev/probes/epi_slack.py [gemm ...]
"""
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
        "ragged": (768, 1000, dict(bias=True, act=2, m=8000)),      # edge tiles in both dimensions
    }
    for name, (Kd, N, ep) in cases.items():
        if only and name not in only:
            continue
        Mr = ep.get("m", M)
        x, w = r(Mr, Kd), r(N, Kd, sc=0.05)
        bias = torch.randn(N, device="cuda") if ep.get("bias") else None
        res = r(Mr, N) if ep.get("res") else None
        aux = torch.empty(Mr, N, device="cuda", dtype=BF) if ep.get("act") else None
        dg = r(Mr, N) if ep.get("dgelu") else None
        fn = lambda: K.gemm_nt_ex(x, w, bias=bias, act=ep.get("act", 0), aux=aux, res=res, dgelu=dg)   # noqa: E731
        out = {"gemm": name, "M": Mr, "N": N, "K": Kd}
        ys = {}
        cfgs = ((0, 0), (1, 0), (0, 1), (1, 1))
        for sl, pr in cfgs:
            o1, o2 = K.tune_set("pp_epi_slack", sl), K.tune_set("pp_epi_pair", pr)
            y = fn()
            torch.cuda.synchronize()
            ys[sl, pr] = (y.clone(), None if aux is None else aux.clone())
            K.tune_set("pp_epi_slack", o1)
            K.tune_set("pp_epi_pair", o2)
        out["same_bits"] = all(torch.equal(ys[0, 0][0], ys[c][0]) and (aux is None or torch.equal(ys[0, 0][1], ys[c][1]))
                               for c in cfgs)
        for rep in range(2):
            for sl, pr in cfgs:
                o1, o2 = K.tune_set("pp_epi_slack", sl), K.tune_set("pp_epi_pair", pr)
                out[f"s{sl}p{pr}_{rep}"] = timeit(fn)
                K.tune_set("pp_epi_slack", o1)
                K.tune_set("pp_epi_pair", o2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
