"""Which hipBLASLt (torch) entry points can serve the framework's PLAIN GEMMs, and how fast, vs the in-tree
engine (the fused-epilogue GEMMs stay on the in-tree MFMA kernels).

For the weight gradients the framework accumulates fp32 dW[N][K] += dY^T[N][M] . X[M][K] from bf16
operands straight into the flat gradient arena, so it needs bf16 x bf16 -> fp32 with beta = 1:
``torch.addmm(c, a, b, out_dtype=torch.float32)`` (torch >= 2.9).  This probes that it exists, accepts an
fp32 ``input`` / ``out`` aliasing it, matches an fp32 reference, and times it against ``gemm_tn_acc``.

    python tools/blas_probe.py            # one JSON line per shape
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_nn_amd.ops import kernels as K  # noqa: E402

BF = torch.bfloat16

# (name, M tokens, N out, K in): the linears of GPT-2 small at B*T = 8192 and its tied LM head
SHAPES = [("qkv", 8192, 2304, 768), ("proj", 8192, 768, 768), ("fc", 8192, 3072, 768), ("fc2", 8192, 768, 3072),
          ("head", 8192, 50304, 768)]


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
    torch.manual_seed(0)
    for name, M, N, Kd in SHAPES:
        r = {"shape": name, "M": M, "N": N, "K": Kd}
        x = torch.randn(M, Kd, device="cuda").to(BF)          # activations [tokens][in]
        g = torch.randn(M, N, device="cuda").to(BF)           # output grads [tokens][out]
        w = torch.randn(N, Kd, device="cuda").to(BF)          # weight [out][in]
        fl = 2.0 * M * N * Kd
        ref = g.float().t() @ x.float()
        # --- weight gradient: fp32 accumulate
        dw = torch.ones(N, Kd, device="cuda")
        try:
            torch.addmm(dw, g.t(), x, out_dtype=torch.float32, out=dw)
            err = ((dw - 1.0 - ref).abs().max() / ref.abs().max()).item()
            r["addmm_out_dtype_inplace_err"] = err
            r["addmm_out_dtype_inplace_tf"] = fl / timeit(lambda: torch.addmm(dw, g.t(), x, out_dtype=torch.float32,
                                                                                out=dw)) / 1e9
        except Exception as e:      # noqa: BLE001
            r["addmm_out_dtype_inplace_error"] = repr(e)[:200]
        try:
            t = torch.mm(g.t(), x, out_dtype=torch.float32)
            r["mm_out_dtype_err"] = ((t - ref).abs().max() / ref.abs().max()).item()
            r["mm_out_dtype_plus_add_tf"] = fl / timeit(lambda: dw.add_(torch.mm(g.t(), x, out_dtype=torch.float32))) / 1e9
        except Exception as e:      # noqa: BLE001
            r["mm_out_dtype_error"] = repr(e)[:200]
        r["ours_tn_acc_tf"] = fl / timeit(lambda: K.gemm_tn_acc(g, x, dw)) / 1e9
        # --- data gradient dX = dY . W (plain, bf16 out)
        r["torch_dgrad_tf"] = fl / timeit(lambda: g @ w) / 1e9
        r["ours_dgrad_tf"] = fl / timeit(lambda: K.gemm_nt_ex(g, w, w_kn=True)) / 1e9
        # --- forward Y = X . W^T (plain)
        r["torch_fwd_tf"] = fl / timeit(lambda: x @ w.t()) / 1e9
        r["ours_fwd_tf"] = fl / timeit(lambda: K.gemm_nt_ex(x, w)) / 1e9
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del x, g, w, dw, ref


if __name__ == "__main__":
    main()
