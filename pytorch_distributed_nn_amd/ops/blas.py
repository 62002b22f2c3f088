"""GEMM engine selection for the transformer linears: hand-written MFMA kernels or hipBLASLt.

The fused-epilogue GEMMs of the GPT-2 block (``kernels.gemm_nt_ex``: bias, GELU with the pre-activation
saved, residual add, dGELU; ``kernels.gemm_tn_acc``: fp32 weight-gradient accumulation straight into the
flat gradient arena) are this framework's own CDNA4 kernels.  For large *plain* GEMM cores hipBLASLt's
tuned assembly is measurably faster on MI355X at the GPT-2 shapes (profiles/blas_probe_r1.jsonl; tokens
M = 8192, K = 768 ... 3072):

    shape (M,N,K)         fwd TF/s ours / hipBLASLt   dgrad ours / hipBLASLt   wgrad(+=, fp32) ours / hipBLASLt
    qkv  8192x2304x768          369 / 782                  517 / 725                 330 / 413
    fc   8192x3072x768          484 / 835                  568 / 834                 391 / 480
    fc2  8192x768x3072          608 / 1011                 438 / 797                 390 / 481
    head 8192x50304x768         623 / 1141                 656 / 1110                677 / 908
    proj 8192x768x768           400 / 488                  383 / 493                 206 / 184

so ``auto`` (the default) runs the GEMM core of those calls on hipBLASLt (through ``torch.mm`` /
``torch.addmm``; bias in the library epilogue, fp32 ``out_dtype`` accumulation in place into the arena
for weight gradients) and keeps the non-GEMM part of each fused epilogue on our kernels (GELU / dGELU
``act`` kernels, residual add).  Everything small, and every convolution, stays on the in-tree MFMA
engines.  ``PDNN_GEMM=mfma`` forces the in-tree kernels everywhere (``blas`` forces the library).

This is a per-call choice on the host (shapes only), so it is stable across steps and safe under hipGraph
capture.
"""
from __future__ import annotations

import os

import torch

from . import kernels as K
from .functional import weight_bf16

BF16 = torch.bfloat16
F32 = torch.float32

MODE = os.environ.get("PDNN_GEMM", "auto").lower()      # auto | mfma | blas


def set_mode(mode: str):
    global MODE
    assert mode in ("auto", "mfma", "blas"), mode
    MODE = mode


def _blas(tokens: int, n: int, k: int, kind: str) -> bool:
    if MODE == "mfma":
        return False
    if MODE == "blas":
        return True
    if tokens < 2048 or min(n, k) < 256:
        return False
    if kind == "wgrad":                       # the square 768x768 projection wgrad is ours (measured)
        return n * k >= 1 << 21
    return True


def linear_fwd(x, wk, bias=None, act=0, aux=None, res=None):
    """y = act(x @ wk^T + bias) (+ res), bf16 [M][N]; with act == 2 (GELU) ``aux`` receives the
    pre-activation.  Same contract as :func:`kernels.gemm_nt_ex`."""
    M, Kd = x.shape
    N = wk.shape[0]
    if not _blas(M, N, Kd, "fwd"):
        return K.gemm_nt_ex(x, wk, bias=bias, act=act, aux=aux, res=res)
    # bf16 bias for the library epilogue: the flat arena's bf16 shadow of the parameter (refreshed by the
    # fused optimizer) instead of a per-call fp32 -> bf16 conversion kernel
    b = weight_bf16(bias) if bias is not None else None
    if act:
        u = aux if aux is not None else torch.empty(M, N, device=x.device, dtype=BF16)
        if b is not None:
            torch.addmm(b, x, wk.t(), out=u)
        else:
            torch.mm(x, wk.t(), out=u)
        y = K.act_fwd(u, "gelu" if act == 2 else "relu")
    else:
        y = torch.addmm(b, x, wk.t()) if b is not None else torch.mm(x, wk.t())
    if res is not None:
        y.add_(res)
    return y


def linear_dgrad(g, wk, dgelu=None):
    """dX = g @ wk (wk stored [N][K] as in the forward); with ``dgelu`` = pre-activation u: dX *= gelu'(u)."""
    M, N = g.shape
    Kd = wk.shape[1]
    if not _blas(M, Kd, N, "dgrad"):
        return K.gemm_nt_ex(g, wk, dgelu=dgelu, w_kn=True)
    d = torch.mm(g, wk)
    if dgelu is not None:
        d = K.act_bwd(d, dgelu, "gelu")
    return d


def wgrad_acc(g, x, out):
    """out[N][K] (fp32) += g[M][N]^T @ x[M][K]."""
    M, N = g.shape
    Kd = x.shape[1]
    if not _blas(M, N, Kd, "wgrad") or not out.is_contiguous():
        return K.gemm_tn_acc(g, x, out)
    torch.addmm(out, g.t(), x, out_dtype=F32, out=out)
    return out
