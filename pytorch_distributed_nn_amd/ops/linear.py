"""Transformer linear layers on the in-tree GEMM engines (no vendor BLAS on any path).

Every call lands in ``csrc/kernels``:

* forward ``y = act(x W^T + b) (+ res)`` and data gradient ``dX = g W (* gelu'(u))`` go through
  ``kernels.gemm_nt_ex``; large shapes run the ping-pong engine (``csrc/kernels/gemm_pp.hip``: 256-row
  tiles, tile width chosen from 96/128/192/256/288 so the grid fills the 256 CUs in whole rounds, glds ring
  with counted vmcnt, fused bias / GELU (+ pre-activation) / dGELU / residual epilogues), small ones the
  128-row register-staged kernel;
* the weight gradient ``dW += g^T x`` (fp32, in place in the flat gradient arena) runs the ping-pong
  engine with both operands reduction-major and split-K partial slabs reduced by a second kernel
  (``kernels.pp_wgrad``), or the glds engine's split-K atomics for shapes it does not take; the bias gradient
  (column sums of g) rides along as row sums of the same MFMA operand (one extra MFMA per fragment against a
  ones fragment) instead of a separate column-sum pass over g.

Reference GEMM sites this replaces: MPI_code/src/util/util.h:35-81 (cblas_dgemm),
MPI_code/src/nn/nn_layer.h:111-175 (forward, dgrad, wgrad of the bias-folded dense layer).
"""
from __future__ import annotations

import torch

from . import kernels as K
from .functional import weight_bf16_t

F32 = torch.float32


def linear_fwd(x, wk, bias=None, act=0, aux=None, res=None):
    """y = act(x @ wk^T + bias) (+ res), bf16 [M][N]; with act == 2 (GELU) ``aux`` receives the
    pre-activation.  Same contract as :func:`kernels.gemm_nt_ex`."""
    return K.gemm_nt_ex(x, wk, bias=bias, act=act, aux=aux, res=res)


def linear_dgrad(g, wk, dgelu=None, p=None):
    """dX = g @ wk (wk stored [N][K] as in the forward); with ``dgelu`` = pre-activation u: dX *= gelu'(u).

    With the parameter ``p`` given, the GEMM reads the cached transposed copy W^T [K][N] (K-major B: every
    tile width of the ping-pong engine is available, measured faster than the reduction-major B form at
    all GPT-2 shapes), and a reduction much longer than the output (the tied LM head: N = vocabulary)
    splits K over work items with fp32 partial slabs."""
    if p is None or not g.is_cuda:
        return K.gemm_nt_ex(g, wk, dgelu=dgelu, w_kn=True)
    wt = weight_bf16_t(p)
    M, N = g.shape
    if dgelu is None and N >= 16384 and N % 32 == 0 and N >= 8 * wt.shape[0]:
        return K.gemm_nt_splitk(g, wt)
    return K.gemm_nt_ex(g, wt, dgelu=dgelu)


def wgrad_acc(g, x, out, bias=None, plan_cus=0):
    """out[N][K] (fp32) += g[M][N]^T @ x[M][K]; with ``bias`` (fp32 [N]) also bias += column sums of g when the
    ping-pong engine runs the product (fused: one extra MFMA per g fragment).  Returns whether ``bias`` was
    accumulated (the caller sums it otherwise).  ``plan_cus``: see kernels.pp_wgrad."""
    M, N = g.shape
    Kd = x.shape[1]
    if M % 32 == 0 and N % 8 == 0 and Kd % 8 == 0 and out.is_contiguous() and M * N * Kd >= (1 << 24):
        K.pp_wgrad(g, x, out, rowsum=bias, plan_cus=plan_cus)
        return bias is not None
    K.gemm_tn_acc(g, x, out)
    return False
