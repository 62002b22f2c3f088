"""Autograd-level ops of the framework.

GPU tensors run the hand-written HIP kernels (``ops.kernels``); CPU tensors run the PyTorch fp32
reference of the same op (that is what the CPU test-suite exercises and what the GPU numerics tests
compare the kernels against).  Activations on the GPU path are NHWC bf16; on the CPU path the
conv/pool ops take NHWC too and compute through NCHW torch ops, so the module code is identical.

Weights are fp32 ``nn.Parameter``s (the optimizer's master copy).  Kernels read a bf16 "shadow" of each
weight in the layout they want (conv: [K][R][S][C]); the fused optimizer refreshes shadows in the same
pass that updates the master weights (see ``optim/``), and :func:`weight_bf16` re-casts on the fly if a
weight was modified outside (detected through the tensor version counter).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..optim import flat
from ..optim.flat import await_param, direct_grad, grad_ready
from . import kernels as K

BF16 = torch.bfloat16


# ------------------------------------------------------------------------------------------------
# weight shadows
# ------------------------------------------------------------------------------------------------
def weight_bf16(p: torch.Tensor, krsc: bool = False) -> torch.Tensor:
    """bf16 copy of parameter ``p`` for the kernels ([K][R][S][C] for 4-D conv weights if krsc)."""
    await_param(p)
    sh = getattr(p, "_pdnn_shadow", None)
    if sh is not None and getattr(p, "_pdnn_shadow_ver", None) == p._version:
        return sh
    src = p.detach()
    if krsc and src.dim() == 4:
        src = src.permute(0, 2, 3, 1)
    out = src.to(BF16).contiguous()
    flat.SHADOW_EPOCH[0] += 1          # a mid-forward re-cast on the compute stream (see flat.SHADOW_EPOCH)
    if sh is not None and sh.shape == out.shape:
        sh.copy_(out)
        p._pdnn_shadow_ver = p._version
        return sh
    return out


def weight_bf16_t(p: torch.Tensor) -> torch.Tensor:
    """bf16 transposed copy W^T [K][N] of a 2-D weight W [N][K] (the data-gradient GEMM's K-major B operand),
    cached per parameter version / flat-arena update generation, rebuilt by the in-tree transpose kernel."""
    await_param(p)                     # before the cache check: a PS bucket landing bumps the generation
    ver = _t_version(p)
    st = getattr(p, "_pdnn_shadow_t", None)
    if st is not None and st[0] == ver:
        tok = p.__dict__.get("_pdnn_t_wait")
        if tok is not None:            # made on the side stream by prefetch_weight_t
            if not tok[1]:
                torch.cuda.current_stream(p.device).wait_event(tok[0])
                tok[1] = True
            p._pdnn_t_wait = None
        return st[1]
    wb = weight_bf16(p)
    if wb.is_cuda:
        out = st[1] if st is not None and st[1].shape == (wb.shape[1], wb.shape[0]) else None
        wt = K.transpose_bf16(wb, out=out)
    else:
        wt = wb.t().contiguous()
    p._pdnn_shadow_t = (ver, wt)
    return wt


def _t_version(p):
    fp = getattr(p, "_pdnn_flat", None)
    return (p._version, fp.generation if fp is not None else 0)


def prefetch_weight_t(ps, side=None):
    """Refresh the transposed copies (:func:`weight_bf16_t`) of every stale 2-D weight of ``ps`` in ONE
    batched launch (``kernels.transpose_bf16_multi``) at the start of a forward, on the ``side`` stream when
    given (ordered after the compute stream's optimizer step; the first backward use waits on one event), so
    the ~50 per-weight ~5 us transposes of a GPT-2 step leave the backward.  Parameters still arriving (PS
    workers mark them ``_pdnn_weight_pending``) keep the lazy per-use path."""
    todo = []
    for p in ps:
        if not p.is_cuda or p.dim() != 2 or "_pdnn_weight_pending" in p.__dict__:
            continue
        ver = _t_version(p)
        st = getattr(p, "_pdnn_shadow_t", None)
        if st is not None and st[0] == ver:
            continue
        wb = weight_bf16(p)
        if not wb.is_contiguous():
            continue
        out = st[1] if st is not None and st[1].shape == (wb.shape[1], wb.shape[0]) else None
        if out is None:
            out = torch.empty(wb.shape[1], wb.shape[0], device=wb.device, dtype=BF16)
        todo.append((p, ver, wb, out))
    if not todo:
        return
    pairs = [(wb, out) for _, _, wb, out in todo]
    if side is None:
        K.transpose_bf16_multi(pairs)
        tok = None
    else:
        main = torch.cuda.current_stream(todo[0][0].device)
        K.stream_wait(side, main)
        with torch.cuda.stream(side):
            K.transpose_bf16_multi(pairs)
            ev = torch.cuda.Event()
            ev.record(side)
        tok = [ev, False]
        for _, _, wb, out in todo:
            out.record_stream(side)
            wb.record_stream(side)
    for p, ver, _, out in todo:
        p._pdnn_shadow_t = (ver, out)
        p._pdnn_t_wait = tok


def _pad_last(t, mult=8):
    c = t.shape[-1]
    pc = (c + mult - 1) // mult * mult
    if pc == c:
        return t
    return F.pad(t, (0, pc - c))


# ------------------------------------------------------------------------------------------------
# Convolution (generic, NHWC)
# ------------------------------------------------------------------------------------------------
class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, wk, stride, padding):
        y, _ = K.conv_fwd(x, wk, stride, padding)
        ctx.save_for_backward(x, wk)
        ctx.conf = (stride, padding, weight.shape)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, wk = ctx.saved_tensors
        st, pad, wshape = ctx.conf
        gy = gy.contiguous()
        Kc, R, S, C = wk.shape
        dx = K.conv_dgrad(gy, wk, x.shape, st, pad) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dwk = K.conv_wgrad(x, gy, R, S, st, pad)           # fp32 [K][R][S][C(padded)]
            Ko, Ci = wshape[0], wshape[1]
            dw = dwk[:Ko, :, :, :Ci].permute(0, 3, 1, 2)     # -> [K][C][R][S] (channels_last strides)
        return dx, dw, None, None, None


def conv2d_nhwc(x, weight, stride=1, padding=0, bias=None):
    """2-D convolution on an NHWC activation.  ``weight`` is the torch-layout [K][C][R][S] parameter.

    GPU: channel counts not divisible by 8 (LeNet's 1/20/50) are zero-padded on the fly; the output
    then keeps its padded channel count (padding channels are exactly zero)."""
    if not x.is_cuda:
        y = F.conv2d(x.permute(0, 3, 1, 2), weight[:, : x.shape[3]] if weight.shape[1] != x.shape[3] else weight,
                     bias, stride, padding)
        return y.permute(0, 2, 3, 1)
    Kc, Cin, R, S = weight.shape
    wk = weight_bf16(weight, krsc=True)
    C = x.shape[3]
    if C != Cin or Kc % 8:
        Kp = (Kc + 7) // 8 * 8
        wk = F.pad(wk, (0, C - Cin, 0, 0, 0, 0, 0, Kp - Kc)).contiguous()
    y = _Conv2dNHWC.apply(x.contiguous(), weight, wk, stride, padding)
    if bias is not None:
        bp = F.pad(bias, (0, y.shape[3] - Kc)) if y.shape[3] != Kc else bias
        y = y + bp.to(BF16)
    return y


# ------------------------------------------------------------------------------------------------
# BatchNorm (generic NHWC, optional fused ReLU)
# ------------------------------------------------------------------------------------------------
class _BatchNormNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, rm, rv, training, momentum, eps, relu):
        N, H, W, C = x.shape
        x2 = x.reshape(-1, C)
        if training:
            slab, rows = K.bn_stats(x2)
            mean, inv, sc, sh = K.bn_finalize(slab, rows, x2.shape[0], eps, momentum, gamma, beta, rm, rv)
        else:
            sc, sh = K.bn_eval_coeff(eps, gamma, beta, rm, rv)
            mean, inv = rm, torch.rsqrt(rv + eps)
        y = K.bn_apply(x2, sc, sh, relu=relu).view_as(x)
        ctx.save_for_backward(x2, y.reshape(-1, C), gamma, mean, inv, sc)
        ctx.conf = (training, relu)
        return y

    @staticmethod
    def backward(ctx, gy):
        x2, y2, gamma, mean, inv, sc = ctx.saved_tensors
        training, relu = ctx.conf
        g2 = gy.contiguous().reshape(x2.shape)
        mode = 1 if relu else 0
        if training:
            slab, _, rows = K.bn_bwd_reduce(g2, x2, mean, inv, mode=mode, msrc=y2)
            dgamma, dbeta = K.bn_bwd_finalize(slab, rows)
            dx, _, _ = K.bn_bwd_apply(g2, x2, mean, inv, gamma, dgamma, dbeta, mode=mode, msrc=y2)
        else:
            gm = g2 if not relu else g2 * (y2 > 0)
            xh = (x2.float() - mean) * inv
            dgamma = (gm.float() * xh).sum(0)
            dbeta = gm.float().sum(0)
            dx = (gm.float() * sc).to(BF16)
        return dx.view(gy.shape), dgamma, dbeta, None, None, None, None, None, None


def batch_norm_nhwc(x, bn: torch.nn.BatchNorm2d, relu=False):
    training = bn.training or bn.running_mean is None
    if not x.is_cuda:
        y = F.batch_norm(x.permute(0, 3, 1, 2), bn.running_mean, bn.running_var, bn.weight, bn.bias, training,
                         bn.momentum if bn.momentum is not None else 0.1, bn.eps)
        y = y.permute(0, 2, 3, 1)
        if training and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
        return F.relu(y) if relu else y
    C = bn.num_features
    if x.shape[3] != C:   # padded channels (LeNet-style) -> pad the affine params
        pc = x.shape[3] - C
        gamma, beta = F.pad(bn.weight, (0, pc), value=1.0), F.pad(bn.bias, (0, pc))
        rm, rv = F.pad(bn.running_mean, (0, pc)), F.pad(bn.running_var, (0, pc), value=1.0)
    else:
        gamma, beta, rm, rv = bn.weight, bn.bias, bn.running_mean, bn.running_var
    if training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    return _BatchNormNHWC.apply(x.contiguous(), gamma, beta, rm, rv, training,
                                bn.momentum if bn.momentum is not None else 0.1, bn.eps, relu)


# ------------------------------------------------------------------------------------------------
# Linear
# ------------------------------------------------------------------------------------------------
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x2, weight, bias, wk, relu):
        y = K.gemm_nt(x2, wk, bias=bias, relu=relu)
        ctx.save_for_backward(x2, wk, y if relu else None)
        ctx.conf = (bias is not None, relu, weight.shape)
        # unpadded weight/bias: their gradients can be accumulated straight into the flat arena
        ctx.direct = (weight, bias) if wk.shape == weight.shape else None
        return y

    @staticmethod
    def backward(ctx, gy):
        x2, wk, y = ctx.saved_tensors
        has_bias, relu, wshape = ctx.conf
        gy = gy.contiguous()
        if relu:
            gy = K.act_bwd(gy, y, "relu")
        dx = K.gemm_nn(gy, wk) if ctx.needs_input_grad[0] else None
        dw = db = None
        direct, ctx.direct = ctx.direct, None
        ready = []
        if ctx.needs_input_grad[1]:
            tw = direct_grad(direct[0]) if direct is not None else None
            if tw is not None:
                K.gemm_tn_acc(gy, x2, tw)
                ready.append(direct[0])
            else:
                dw = torch.zeros(wk.shape, device=gy.device, dtype=torch.float32)
                K.gemm_tn_acc(gy, x2, dw)
                dw = dw[: wshape[0], : wshape[1]]
        if has_bias and ctx.needs_input_grad[2]:
            tb = direct_grad(direct[1]) if direct is not None else None
            if tb is not None:
                K.colsum(gy, out=tb, accumulate=True)
                ready.append(direct[1])
            else:
                db = K.colsum(gy)              # shape of the (possibly padded) bias input
        for p in ready:
            grad_ready(p)
        return dx, dw, db, None, None


def linear(x, weight, bias=None, relu=False):
    """y = x W^T + b (optionally fused ReLU).  GPU: bf16 in/out, fp32 accumulate."""
    if not x.is_cuda:
        y = F.linear(x, weight, bias)
        return F.relu(y) if relu else y
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    if x2.dtype != BF16:
        x2 = x2.to(BF16)
    N, Kd = weight.shape
    wk = weight_bf16(weight)
    Np, Kp = (N + 7) // 8 * 8, (Kd + 7) // 8 * 8
    b = bias
    if Np != N or Kp != Kd:
        wk = F.pad(wk, (0, Kp - Kd, 0, Np - N)).contiguous()
        b = F.pad(bias, (0, Np - N)) if bias is not None else None
    if x2.shape[1] != Kp:
        x2 = F.pad(x2, (0, Kp - x2.shape[1]))
    x2 = x2.contiguous()
    y = _Linear.apply(x2, weight, b, wk, relu)
    if Np != N:
        y = y[:, :N]
    return y.reshape(*shp[:-1], N)


# ------------------------------------------------------------------------------------------------
# Activations / elementwise
# ------------------------------------------------------------------------------------------------
class _Act(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, op):
        y = K.act_fwd(x, op)
        ctx.save_for_backward(x)
        ctx.op = op
        return y

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return K.act_bwd(g, x, ctx.op), None


def _act(x, op, ref):
    if not x.is_cuda or x.numel() % 8 or x.dtype != BF16:
        return ref(x)
    return _Act.apply(x.contiguous(), op)


def relu(x):
    return _act(x, "relu", F.relu)


def sigmoid(x):
    return _act(x, "sigmoid", torch.sigmoid)


def gelu(x):
    return _act(x, "gelu", lambda t: F.gelu(t, approximate="tanh"))


# ------------------------------------------------------------------------------------------------
# Pooling (NHWC)
# ------------------------------------------------------------------------------------------------
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, st, pad):
        y, idx = K.maxpool_fwd(x, k, st, pad)
        ctx.save_for_backward(idx)
        ctx.conf = (x.shape, k, st, pad)
        return y

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        shape, k, st, pad = ctx.conf
        return K.maxpool_bwd(g, idx, shape, k, st, pad), None, None, None


def max_pool2d_nhwc(x, k, stride=None, padding=0):
    stride = stride or k
    if not x.is_cuda:
        return F.max_pool2d(x.permute(0, 3, 1, 2), k, stride, padding).permute(0, 2, 3, 1)
    return _MaxPool.apply(x.contiguous(), k, stride, padding)


class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shape = x.shape
        return K.avgpool_fwd(x)

    @staticmethod
    def backward(ctx, g):
        return K.avgpool_bwd(g, ctx.shape)


def global_avg_pool_nhwc(x):
    """[N,H,W,C] -> [N,C] mean over H, W."""
    if not x.is_cuda:
        return x.mean(dim=(1, 2))
    return _GAP.apply(x.contiguous())


def avg_pool2d_nhwc(x, k):
    """avg_pool2d with kernel == spatial size (the reference's F.avg_pool2d(out, 4) at 4x4)."""
    if x.shape[1] == k and x.shape[2] == k:
        return global_avg_pool_nhwc(x).reshape(x.shape[0], 1, 1, x.shape[3])
    return F.avg_pool2d(x.permute(0, 3, 1, 2), k).permute(0, 2, 3, 1)


# ------------------------------------------------------------------------------------------------
# Cross entropy (fused softmax + NLL)
# ------------------------------------------------------------------------------------------------
class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, reduction):
        loss, lse, acc = K.xent_fwd(logits, target, ignore_index)
        ctx.save_for_backward(logits, target, lse, acc)
        ctx.conf = (ignore_index, reduction)
        if reduction == "sum":
            return acc[0].clone()
        if reduction == "none":
            return loss
        return acc[0] / acc[1].clamp_min(1.0)

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, acc = ctx.saved_tensors
        ignore_index, reduction = ctx.conf
        if reduction == "none":
            # per-row scale: fold into labels-independent path (rare; small tensors)
            p = torch.softmax(logits.float(), -1)
            p[torch.arange(p.shape[0], device=p.device), target.clamp_min(0)] -= 1
            p = p * (target != ignore_index).unsqueeze(1) * g.unsqueeze(1)
            return p.to(logits.dtype), None, None, None
        gs = g.reshape(1)
        if gs.dtype != torch.float32:
            gs = gs.float()
        d = K.xent_bwd(logits, target, lse, gs, 1.0, ignore_index, count=acc[1:2] if reduction == "mean" else None)
        return d, None, None, None


def cross_entropy(logits, target, ignore_index=-100, reduction="mean"):
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target, ignore_index=ignore_index, reduction=reduction)
    lg = logits.reshape(-1, logits.shape[-1])
    if lg.dtype not in (BF16, torch.float32):
        lg = lg.float()
    return _XEnt.apply(lg.contiguous(), target.reshape(-1).long().contiguous(), ignore_index, reduction)


# ------------------------------------------------------------------------------------------------
# input layout
# ------------------------------------------------------------------------------------------------
def nchw_to_nhwc_input(x, cpad=None):
    """Data-loader NCHW batch -> NHWC activation (GPU: bf16, channels zero-padded to a multiple of 8)."""
    if not x.is_cuda:
        return x.permute(0, 2, 3, 1).float()
    C = x.shape[1]
    cp = cpad or (C + 7) // 8 * 8
    return K.nchw_to_nhwc(x, cp)
