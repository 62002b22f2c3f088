"""Fused GPT-2 building blocks (BASELINE.json config 4: "GPT-2-small transformer DDP bf16 8xMI355X
(LayerNorm + attention GEMM HIP kernels)").  The reference has no transformer (SURVEY.md §2 lists CNNs and
MLPs only), so this is new capability exercising the same engine: every GEMM runs on the MFMA engine of
``csrc/kernels/gemm_mfma.hip`` and every row op on ``csrc/kernels/transformer.hip``.

A whole pre-LN block ``x + attn(ln_1(x))`` -> ``+ mlp(ln_2(.))`` is ONE autograd Function
(:class:`GPT2BlockFn`) so the backward schedules its own kernels (fused epilogues, no autograd glue):

forward                                              backward
  ln1 = LN(x)                 layernorm_fwd            dh   = dx2 . Wfc2 * gelu'(u)   gemm_nt_ex (w_kn, dgelu epilogue)
  qkv = ln1 Wqkv^T + b        gemm_nt_ex(bias)         dWfc2 += dx2^T h ; dbfc2 = colsum(dx2)
  S   = Q K^T (per b, h)      gemm_batched(causal=1)   dln2 = dh . Wfc ; dWfc, dbfc
  P   = softmax(S/sqrt(d))    attn_softmax_fwd         dx1  = LN2_bwd(dln2) + dx2     (residual fused)
  y   = P V                   gemm_batched(causal=2)   dy   = dx1 . Wproj ; dWproj, dbproj
  x1  = x + y Wproj^T + b     gemm_nt_ex(res=x)        attention bwd (dV, dP, dS, dQ, dK: 4 batched GEMMs
  ln2 = LN(x1)                                               + attn_softmax_bwd), written into dqkv
  h   = gelu(ln2 Wfc^T + b)   gemm_nt_ex(GELU, aux=u)  dln1 = dqkv . Wqkv ; dWqkv, dbqkv
  x2  = x1 + h Wfc2^T + b     gemm_nt_ex(res=x1)       dx   = LN1_bwd(dln1) + dx1

The residual stream is bf16 [B*T][D]; LayerNorm statistics, GEMM accumulation, softmax and all weight
gradients are fp32.  Attention (head dim 64, T % 128 == 0) runs the fused flash kernels of
``csrc/kernels/attention.hip`` (scores never leave registers; backward recomputes P from the saved
log-sum-exp); other shapes fall back to the materialised path below (batched MFMA GEMMs with causal tile
skipping + row-softmax kernels).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ..optim.flat import direct_grad, grad_ready
from . import linear as BL
from . import kernels as K
from .. import tuning as _tuning

BF16 = torch.bfloat16
F32 = torch.float32


# ------------------------------------------------------------------------------------------------
# attention core on a packed qkv [B*T][3D] bf16 tensor
# ------------------------------------------------------------------------------------------------
def attention_fwd(qkv, B, T, H, causal=True):
    """-> y [B*T][D] bf16, P [B*H*T][T] bf16 (saved for backward)."""
    D = qkv.shape[1] // 3
    d = D // H
    ld = 3 * D
    dev = qkv.device
    S = torch.empty(B * H * T, T, device=dev, dtype=F32)
    P = torch.empty(B * H * T, T, device=dev, dtype=BF16)
    lse = torch.empty(B * H * T, device=dev, dtype=F32)
    y = torch.empty(B * T, D, device=dev, dtype=BF16)
    q, k, v = qkv, qkv[:, D:], qkv[:, 2 * D:]
    # S[b,h] = Q K^T : A = Q [T][d] (K-major), B = K [T][d] (K-major)
    K.gemm_batched(q, ld, (T * ld, d), 0, k, ld, (T * ld, d), 0, S, T, (H * T * T, T * T), T, T, d, (B, H),
                   causal=1 if causal else 0)
    K.attn_softmax_fwd(S, P, lse, B * H * T, T, 1.0 / math.sqrt(d), causal)
    # y[b, :, h] = P V : A = P [T][T], B = V stored [T(k)][d]
    K.gemm_batched(P, T, (H * T * T, T * T), 0, v, ld, (T * ld, d), 1, y, D, (T * D, d), T, d, T, (B, H),
                   causal=2 if causal else 0)
    return y, P, S


def attention_bwd(dy, qkv, P, B, T, H, causal=True, dS_buf=None):
    """dy [B*T][D] -> dqkv [B*T][3D].  ``dS_buf``: fp32 [B*H*T][T] scratch (the forward's S)."""
    D = qkv.shape[1] // 3
    d = D // H
    ld = 3 * D
    dev = qkv.device
    dqkv = torch.empty(B * T, ld, device=dev, dtype=BF16)
    q, k, v = qkv, qkv[:, D:], qkv[:, 2 * D:]
    dq, dk, dv = dqkv, dqkv[:, D:], dqkv[:, 2 * D:]
    sP = (H * T * T, T * T)
    # dV = P^T dO : A = P stored [q][k] = [K][M] (amode 1), B = dO stored [q][d] = [K][N] (bmode 1)
    K.gemm_batched(P, T, sP, 1, dy, D, (T * D, d), 1, dv, ld, (T * ld, d), T, d, T, (B, H),
                   causal=3 if causal else 0)
    # dP = dO V^T (fp32)
    dP = dS_buf if dS_buf is not None else torch.empty(B * H * T, T, device=dev, dtype=F32)
    K.gemm_batched(dy, D, (T * D, d), 0, v, ld, (T * ld, d), 0, dP, T, sP, T, T, d, (B, H),
                   causal=1 if causal else 0)
    # dS = P * (dP - rowsum(P dP)) / sqrt(d), written over P (row-local, read-before-write per element)
    dS = P
    K.attn_softmax_bwd(P, dP, dS, B * H * T, T, 1.0 / math.sqrt(d), causal)
    # dQ = dS K : B = K stored [k][d] = [K][N]
    K.gemm_batched(dS, T, sP, 0, k, ld, (T * ld, d), 1, dq, ld, (T * ld, d), T, d, T, (B, H),
                   causal=2 if causal else 0)
    # dK = dS^T Q : A = dS stored [q][k] = [K][M], B = Q stored [q][d] = [K][N]
    K.gemm_batched(dS, T, sP, 1, q, ld, (T * ld, d), 1, dk, ld, (T * ld, d), T, d, T, (B, H),
                   causal=3 if causal else 0)
    return dqkv


def use_flash(T, D, H):
    return D // H == 64 and T % 128 == 0


def attention_reference(qkv, B, T, H, causal=True):
    """fp32 PyTorch reference of :func:`attention_fwd` (tests, CPU path)."""
    D = qkv.shape[1] // 3
    q, k, v = qkv.float().view(B, T, 3, H, D // H).permute(2, 0, 3, 1, 4)
    y = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
    return y.transpose(1, 2).reshape(B * T, D)


# ------------------------------------------------------------------------------------------------
# LayerNorm
# ------------------------------------------------------------------------------------------------
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, weight, bias, eps):
        y, mean, rstd = K.layernorm_fwd(x2, weight, bias, eps)
        ctx.save_for_backward(x2, weight, mean, rstd)
        return y

    @staticmethod
    def backward(ctx, gy):
        x2, weight, mean, rstd = ctx.saved_tensors
        dx, dg, db = K.layernorm_bwd(gy.to(BF16), x2, weight, mean, rstd)
        return dx, dg, db, None


def layer_norm(x, weight, bias, eps=1e-5):
    if not x.is_cuda:
        return F.layer_norm(x, (x.shape[-1],), weight, bias, eps)
    shp = x.shape
    x2 = x.reshape(-1, shp[-1]).to(BF16).contiguous()
    return _LayerNorm.apply(x2, weight, bias, eps).view(shp)


# ------------------------------------------------------------------------------------------------
# embedding (token + position)
# ------------------------------------------------------------------------------------------------
class EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, T, wte_k, wpe_k, wte, wpe, head_direct=False, tail=None):
        ctx.save_for_backward(idx)
        ctx.conf = (T, wte_k.shape, wpe.shape)
        ctx.wpe, ctx.wte = wpe, wte
        ctx.head_direct = head_direct       # the tied LM head accumulates its wte gradient in the arena too
        ctx.tail = tail                     # (ddp, wte): split tied embedding, wte is NOT an input (wte=None)
        return K.embedding_fwd(idx, wte_k, wpe_k, T)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        T, s_te, s_pe = ctx.conf
        if ctx.tail is not None:
            # split tied embedding (parallel/ddp.py reduce_sparse_rows): the LM head's dense gradient was announced
            # (and its bucket all-reduced) at the start of the backward; these B*T rows are gathered from every rank
            # and added on top after it
            ddp, wte = ctx.tail
            ctx.tail = None
            tpe = direct_grad(ctx.wpe)
            dwpe = tpe if tpe is not None else torch.zeros(s_pe, device=g.device, dtype=F32)
            K.embedding_bwd(idx, g, None, dwpe, T)
            if tpe is not None:
                grad_ready(ctx.wpe)
                dwpe = None
            gw = wte.grad
            ddp.reduce_sparse_rows(wte, idx, g, lambda i, r, sc: K.embedding_bwd(i, r, gw, None, T, scale=sc))
            ctx.wpe = ctx.wte = None
            return None, None, None, None, None, dwpe, None, None
        # wte is tied with the LM head, whose backward ran first and (with a flat arena) already accumulated
        # its part in place: the embedding adds its rows on top (atomics) and announces the parameter, so no
        # zero-filled temporaries and no autograd sum of the two gradients
        tte = direct_grad(ctx.wte) if ctx.head_direct else None
        dwte = tte if tte is not None else torch.zeros(s_te, device=g.device, dtype=F32)
        tpe = direct_grad(ctx.wpe)
        dwpe = tpe if tpe is not None else torch.zeros(s_pe, device=g.device, dtype=F32)
        K.embedding_bwd(idx, g, dwte, dwpe, T)
        if tpe is not None:
            grad_ready(ctx.wpe)
            dwpe = None
        if tte is not None:
            grad_ready(ctx.wte)
            dwte = None
        ctx.wpe = ctx.wte = None
        return None, None, None, None, dwte, dwpe, None, None


# ------------------------------------------------------------------------------------------------
# one transformer block
# ------------------------------------------------------------------------------------------------
def _wgrad(g, x, shape):
    dw = torch.zeros(shape, device=g.device, dtype=F32)
    BL.wgrad_acc(g, x, dw)
    return dw


class _Sink:
    """Routes parameter gradients straight into the flat arena when possible (optim.flat.direct_grad):
    the GEMM / column-sum / LayerNorm kernels accumulate in place, the op returns None for the parameter
    and announces it with grad_ready.  Otherwise the gradient is returned to autograd.

    tuning gpt2_side_wgrad: arena-bound weight gradients run on the ResNets' weight-gradient side stream
    (ops/fused_resnet.py) beside the data-gradient chain, joined like theirs (at the end of the backward when
    every hook reading them is side-aware, i.e. DDP's bucket launches)."""

    def __init__(self):
        self.ready = []
        self.side = None
        self.forked = False

    def _tgt(self, p):
        t = direct_grad(p)
        if t is not None:
            self.ready.append(p)
        return t

    def _side(self, g):
        if not _tuning.get("gpt2_side_wgrad") or not g.is_cuda:
            return None
        from .fused_resnet import _side_stream
        return _side_stream(g.device)

    def linear(self, p_w, p_b, g, x):
        tw = self._tgt(p_w)
        tb = self._tgt(p_b) if p_b is not None else None
        bias_in = tb if _tuning.get("bias_in_wgrad") else None
        side = self._side(g) if tw is not None and (p_b is None or tb is not None) else None
        if side is not None:
            main = torch.cuda.current_stream(g.device)
            K.stream_wait(side, main)
            with torch.cuda.stream(side):
                bias_done = BL.wgrad_acc(g, x, tw, bias=bias_in, plan_cus=_tuning.get("wgrad_plan_cus"))
                if p_b is not None and not bias_done:
                    K.colsum(g, out=tb, accumulate=True, deterministic=not _tuning.get("colsum_atomic"))
            for t in (g, x):
                t.record_stream(side)
            self.side, self.forked = side, True
            from .fused_resnet import _FORKS
            _FORKS[g.device.index] = _FORKS.get(g.device.index, 0) + 1
            return None, None
        bias_done = False
        if tw is not None:
            # the bias gradient fused into the weight-gradient GEMM when both land in the arena
            bias_done = BL.wgrad_acc(g, x, tw, bias=bias_in)
            rw = None
        else:
            rw = _wgrad(g, x, p_w.shape)
        rb = None
        if p_b is not None and not bias_done:
            if tb is not None:
                K.colsum(g, out=tb, accumulate=True, deterministic=not _tuning.get("colsum_atomic"))
            else:
                rb = K.colsum(g)
        return rw, rb

    def layernorm(self, dy, x, w, m, r, dres, p_w, p_b):
        tw, tb = direct_grad(p_w), direct_grad(p_b)
        if tw is not None and tb is not None:
            self.ready += [p_w, p_b]
            dx, _, _ = K.layernorm_bwd(dy, x, w, m, r, dres=dres, acc=(tw, tb))
            return dx, None, None
        return K.layernorm_bwd(dy, x, w, m, r, dres=dres)

    def done(self):
        if self.forked:
            self.forked = False
            from .fused_resnet import _join_at_backward_end
            if all(getattr(fn, "_pdnn_side_aware", False) for p in self.ready for fn in getattr(p, "_pdnn_grad_hooks", ())):
                _join_at_backward_end(self.side)
            else:
                K.stream_wait(torch.cuda.current_stream(self.side.device), self.side)
        for p in self.ready:
            grad_ready(p)


class GPT2BlockFn(torch.autograd.Function):
    """params: ln1_w, ln1_b, attn_w, attn_b, proj_w, proj_b, ln2_w, ln2_b, fc_w, fc_b, fc2_w, fc2_b
    shadows: bf16 copies of attn_w [3D][D], proj_w [D][D], fc_w [4D][D], fc2_w [D][4D]."""

    @staticmethod
    def forward(ctx, x, conf, shadows, *params):
        B, T, H, eps = conf[:4]
        metas = conf[4] if len(conf) > 4 else None
        ln1w, ln1b, _, attn_b, _, proj_b, ln2w, ln2b, _, fc_b, _, fc2_b = params
        wqkv, wproj, wfc, wfc2 = shadows
        if metas is not None:
            from .fp8 import linear_fp8_fwd

            def lin(inp, i, wk, **kw):      # forward GEMM on the fp8 engine (weights: params[2/4/8/10])
                return linear_fp8_fwd(inp, params[i], metas[(i - 2) // 2 if i < 6 else (i - 4) // 2], **kw)
        else:
            def lin(inp, i, wk, **kw):
                return BL.linear_fwd(inp, wk, **kw)
        ln1, m1, r1 = K.layernorm_fwd(x, ln1w, ln1b, eps)
        qkv = lin(ln1, 2, wqkv, bias=attn_b)
        D = x.shape[1]
        flash = use_flash(T, D, H)
        if flash:
            y, P = K.flash_attn_fwd(qkv, B, T, H, 1.0 / math.sqrt(D // H))     # P := lse2
            S = None
        else:
            y, P, S = attention_fwd(qkv, B, T, H)
        x1 = lin(y, 4, wproj, bias=proj_b, res=x)
        ln2, m2, r2 = K.layernorm_fwd(x1, ln2w, ln2b, eps)
        u = torch.empty(x.shape[0], wfc.shape[0], device=x.device, dtype=BF16)
        h = lin(ln2, 8, wfc, bias=fc_b, act=2, aux=u)
        x2 = lin(h, 10, wfc2, bias=fc2_b, res=x1)
        ctx.save_for_backward(x, ln1, m1, r1, qkv, P, y, x1, ln2, m2, r2, u, h, ln1w, ln2w, *shadows)
        ctx.conf = conf
        ctx.flash = flash
        ctx.S = S          # materialised path: reused as the fp32 dP scratch in backward
        ctx.params = params
        return x2

    @staticmethod
    def backward(ctx, g):
        (x, ln1, m1, r1, qkv, P, y, x1, ln2, m2, r2, u, h, ln1w, ln2w, wqkv, wproj, wfc, wfc2) = ctx.saved_tensors
        B, T, H, eps = ctx.conf[:4]
        Pm = ctx.params
        ctx.params = None
        sink = _Sink()
        g = g.contiguous()
        if g.is_cuda and _tuning.get("wt_layer_batch"):
            # the four data-gradient GEMMs' transposed weights of this block in one launch, just before use
            from .functional import prefetch_weight_t
            prefetch_weight_t((Pm[10], Pm[8], Pm[4], Pm[2]))
        # MLP
        du = BL.linear_dgrad(g, wfc2, dgelu=u, p=Pm[10])                       # (g . Wfc2) * gelu'(u)
        dfc2_w, dfc2_b = sink.linear(Pm[10], Pm[11], g, h)
        dln2 = BL.linear_dgrad(du, wfc, p=Pm[8])
        dfc_w, dfc_b = sink.linear(Pm[8], Pm[9], du, ln2)
        dx1, dln2w, dln2b = sink.layernorm(dln2, x1, ln2w, m2, r2, g, Pm[6], Pm[7])
        # attention
        dy = BL.linear_dgrad(dx1, wproj, p=Pm[4])
        dproj_w, dproj_b = sink.linear(Pm[4], Pm[5], dx1, y)
        if ctx.flash:
            dqkv = K.flash_attn_bwd(qkv, y, dy, P, B, T, H, 1.0 / math.sqrt(x.shape[1] // H))
        else:
            dqkv = attention_bwd(dy, qkv, P, B, T, H, dS_buf=ctx.S)
        ctx.S = None
        dln1 = BL.linear_dgrad(dqkv, wqkv, p=Pm[2])
        dattn_w, dattn_b = sink.linear(Pm[2], Pm[3], dqkv, ln1)
        dx, dln1w, dln1b = sink.layernorm(dln1, x, ln1w, m1, r1, dx1, Pm[0], Pm[1])
        sink.done()
        return (dx, None, None, dln1w, dln1b, dattn_w, dattn_b, dproj_w, dproj_b, dln2w, dln2b, dfc_w, dfc_b,
                dfc2_w, dfc2_b)


# ------------------------------------------------------------------------------------------------
# final LayerNorm + tied LM head + cross-entropy
# ------------------------------------------------------------------------------------------------
class LMHeadLossFn(torch.autograd.Function):
    """loss = mean CE(LN_f(x) . Wte^T, targets); logits bf16 [B*T][V] live only inside this op."""

    @staticmethod
    def forward(ctx, x, targets, eps, wte_k, lnw, lnb, wte, head_direct=False, split=False, training=False):
        ctx.head_direct = head_direct
        ctx.split = split                   # split tied embedding: the head announces wte itself
        xf, m, r = K.layernorm_fwd(x, lnw, lnb, eps)
        logits = BL.linear_fwd(xf, wte_k)
        # training (grad mode on at the call): the forward also writes the unscaled gradient softmax - onehot over
        # the logits (one read + one write of the 8192 x 50304 logits instead of three passes); the backward then
        # scales the head's 8192 x 768 products by grad_out / count instead of the logits gradient
        ctx.fused = training and _tuning.get("xent_fused") and logits.is_cuda and K.xent_fwd_grad_ok(logits)
        if ctx.fused:
            _, lse, acc, _ = K.xent_fwd_grad(logits, targets)
        else:
            _, lse, acc = K.xent_fwd(logits, targets)
        ctx.save_for_backward(x, xf, m, r, logits, targets, lse, acc, lnw, wte_k)
        ctx.eps = eps
        ctx.params = (lnw, lnb)
        ctx.wte = wte
        return acc[0] / acc[1].clamp_min(1.0)

    @staticmethod
    def backward(ctx, g):
        x, xf, m, r, logits, targets, lse, acc, lnw, wte_k = ctx.saved_tensors
        gs = g.reshape(1)
        if gs.dtype != torch.float32:
            gs = gs.float()
        if ctx.fused:           # logits hold softmax - onehot: scale the products instead (device scalar, no sync)
            dlogits = logits
            sc = gs / acc[1:2].clamp_min(1.0)
            dxf = BL.linear_dgrad(dlogits, wte_k, p=ctx.wte)
            dxf.mul_(sc)
            xf = xf.clone()
            xf.mul_(sc)
        else:
            dlogits = K.xent_bwd(logits, targets, lse, gs, 1.0, count=acc[1:2])
            dxf = BL.linear_dgrad(dlogits, wte_k, p=ctx.wte)
        tte = direct_grad(ctx.wte) if ctx.head_direct else None
        if tte is not None:     # tied weight: the embedding backward adds its part and announces it
            BL.wgrad_acc(dlogits, xf, tte)
            dwte = None
            if ctx.split:       # ... unless its rows are reduced separately: the dense part is complete now
                grad_ready(ctx.wte)
        else:
            dwte = _wgrad(dlogits, xf, wte_k.shape)     # summed with the embedding's by autograd
        sink = _Sink()
        dx, dlnw, dlnb = sink.layernorm(dxf, x, lnw, m, r, None, *ctx.params)
        ctx.params = None
        ctx.wte = None
        sink.done()
        return dx, None, None, None, dlnw, dlnb, dwte, None, None, None
