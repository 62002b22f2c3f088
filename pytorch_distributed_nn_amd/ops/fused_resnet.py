"""Block-level fused ResNet ops for the GPU path (NHWC bf16 activations, fp32 BN statistics).

A whole Bottleneck / BasicBlock / stem is ONE autograd Function whose forward and backward are
hand-scheduled sequences of HIP kernels (reference modules: pytorch_code/model_ops/resnet.py:14-64;
the reference's layer-wise "Split" backward that streams gradients out early, resnet_split.py:235-326,
is replaced by DDP bucket hooks firing as each block's backward completes).

Fusion plan of a Bottleneck (x -> out):

  forward                                          what is written to HBM
  t1 = conv1x1(x)          + BN1 partial stats      t1
  t2 = conv3x3(relu(bn1(t1)))  + BN2 stats          t2       (BN1 + ReLU applied while the halo kernel stages t1;
                                                            a1 materialised only for the implicit-GEMM routes)
  t3 = conv1x1(relu(bn2(t2)))  + BN3 stats           t3       (a2 never materialised)
  td = conv1x1/s(x)        + BNd stats  (if downsample)
  out = relu(bn3(t3) + bnd(td) | x)   one kernel    out

  backward mirrors it: one reduce + one apply kernel per BN (ReLU masks recomputed from t and the BN
  affine, or read from `out`), conv wgrads read the virtual activations relu(bn(t)) through the same
  fused prologue, dgrads are implicit GEMMs on the weight without any transposed copy.
"""
from __future__ import annotations

import contextlib
import os

import torch

from .. import tuning
from ..optim.flat import SHADOW_EPOCH, direct_grad, grad_ready
from . import kernels as K
from .functional import weight_bf16

F32 = torch.float32


def _bn_train(slab, M, bn_params, bufs, mom, eps):
    gamma, beta = bn_params
    rm, rv = bufs
    rows = slab.shape[0] // 2
    return K.bn_finalize(slab, rows, M, eps, mom, gamma, beta, rm, rv)


def _bn_eval(bn_params, bufs, eps):
    gamma, beta = bn_params
    rm, rv = bufs
    sc, sh = K.bn_eval_coeff(eps, gamma, beta, rm, rv)
    return rm, torch.rsqrt(rv + eps), sc, sh


def _conv_bn(x, wk, st, pad, pro, training, bn_params, bufs, mom, eps):
    t, slab = K.conv_fwd(x, wk, st, pad, pro=pro, want_stats=training)
    M = t.numel() // t.shape[-1]
    if training:
        mean, inv, sc, sh = _bn_train(slab, M, bn_params, bufs, mom, eps)
    else:
        mean, inv, sc, sh = _bn_eval(bn_params, bufs, eps)
    return t, mean, inv, sc, sh


_SIDE = {}
# Bottleneck forward: materialise a2 = relu(bn2(t2)) for conv3 (tuning materialize_a2) or apply BN2+ReLU in
# conv3's operand prologue.  Identity-block backward: gout * mask is added by conv1's dgrad epilogue rather
# than materialised by the BN backward (one activation write less per block; +0.2%, gpurun_out/r3_07).
MASKED_RES = True


def side_stream_if_active(t):
    """The side stream that may still be writing weight gradients of `t`'s device, else None."""
    if not t.is_cuda:
        return None
    return _SIDE.get(t.device.index)


def _side_stream(dev):
    """The weight-gradient side stream of a device (tuning side_wgrad = 0 disables it).  It runs at the
    default (lowest) priority; the compute stream gets the high one (bench.py)."""
    if not tuning.get("side_wgrad") or dev.type != "cuda":
        return None
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(device=dev, priority=0)
    return s


class _Sink:
    """Parameter-gradient routing of one fused backward: gradients go straight into the flat arena
    (optim.flat.direct_grad) when possible — the op then returns None for them and announces them with
    grad_ready — otherwise they are returned to autograd.

    Weight gradients run on a side HIP stream: a conv's wgrad (dt, x -> dW) and the data-gradient chain
    (dt -> dgrad -> BN backward -> next dt) are independent, so the split-K wgrad blocks fill the partial
    last rounds of the dgrad grids (and vice versa) instead of each kernel draining the chip on its own.
    Each wgrad is ordered after everything queued on the compute stream so far (its operands); `done()`
    joins the side stream back before the gradients are announced.  The operands stay referenced by the
    block's backward until that join, so the caching allocator cannot hand their memory out early; a
    hipGraph capture records the fork/join as graph edges."""

    def __init__(self, device=None):
        self.ready = []
        self.side = _side_stream(device) if device is not None else None
        self.forked = False
        self.returned = False

    def acc(self, *ps):
        tg = [direct_grad(p) for p in ps]
        if any(t is None for t in tg):
            return None
        self.ready += ps
        return tg

    def bn(self, slab, rows, gamma_p, beta_p):
        """-> (dgamma, dbeta) for bn_bwd_apply, (returned grads of gamma, beta)"""
        acc = self.acc(gamma_p, beta_p)
        dg, db = K.bn_bwd_finalize(slab, rows, acc=acc)
        return (dg, db), ((None, None) if acc is not None else (dg, db))

    def wgrad(self, w_p, x, dy, R, S, st, pad, pro=None, fp8=None):
        if self.side is None:
            return self._wgrad(w_p, x, dy, R, S, st, pad, pro, fp8)
        return self._fork([(w_p, x, dy, R, S, st, pad, pro, fp8)])

    def _fork(self, jobs):
        # (holding a weight gradient back to share the next fork's marker measured neutral: gpurun_out/r3_60)
        main = torch.cuda.current_stream(jobs[0][1].device)
        K.stream_wait(self.side, main)
        self.forked = True
        _FORKS[main.device.index] = _FORKS.get(main.device.index, 0) + 1
        with torch.cuda.stream(self.side):
            gs = [self._wgrad(*j) for j in jobs]
        # the side stream may still read the operands after this block's backward returned (deferred join):
        # the caching allocator must not hand their memory to the compute stream before that work is done
        for j in jobs:
            pro = j[7]
            for t in (j[1], j[2]) + (tuple(pro) if pro is not None else ()):
                t.record_stream(self.side)
        g = gs[-1]
        if g is not None:
            g.record_stream(main)        # allocated on the side stream, consumed by autograd on the main one
            self.returned = True
        return g

    def _wgrad(self, w_p, x, dy, R, S, st, pad, pro, fp8=None):
        acc = self.acc(w_p)
        if fp8 is not None:          # fp8 conv2 (Fp8Conv2): both operands' scales are current for x and dy
            if acc is not None:
                K.conv3x3_wgrad_fp8(x, dy, fp8.fwd, fp8.bwd, out=acc[0].permute(0, 2, 3, 1), pro=pro)
                return None
            return _krsc_grad(K.conv3x3_wgrad_fp8(x, dy, fp8.fwd, fp8.bwd, pro=pro))
        if acc is not None:
            K.conv_wgrad(x, dy, R, S, st, pad, pro=pro, out=acc[0].permute(0, 2, 3, 1))
            return None
        return _krsc_grad(K.conv_wgrad(x, dy, R, S, st, pad, pro=pro))

    def done(self):
        if self.forked:
            self.forked = False
            if self.returned or not all(getattr(fn, "_pdnn_side_aware", False)
                                        for p in self.ready for fn in getattr(p, "_pdnn_grad_hooks", ())):
                # gradients consumed now (autograd, or grad-ready hooks that read them on the compute
                # stream): join before announcing them.  Side-aware hooks (DDP bucket launches) order their
                # collectives after the side stream themselves (side_stream_if_active), so the compute
                # stream is not held up.
                K.stream_wait(torch.cuda.current_stream(self.side.device), self.side)
            else:
                # nothing reads them before the optimizer: join once at the end of the backward, so a block's
                # last weight gradients also overlap the next block's data-gradient chain
                _join_at_backward_end(self.side)
        for p in self.ready:
            grad_ready(p)


_FORKS = {}       # device index -> weight-gradient forks issued so far
_JOINED = {}      # device index -> forks covered by the last end-of-backward join


def _join_at_backward_end(side):
    # one callback per block (not a shared "already queued" flag, which an aborted backward would leave set);
    # the first to run joins every fork issued so far, the rest find nothing new and add no marker (the
    # callbacks all run after the last backward node, so the first join covers them all; one join per block
    # instead: -0.3%, gpurun_out/r3_60).  A final callback runs with backward()'s caller stream current (the
    # stream the optimizer step follows on: tools/callback_stream_probe.py, gpurun_out/r3_64)
    dev = side.device.index

    def join():
        n = _FORKS.get(dev, 0)
        if _JOINED.get(dev) == n:
            return
        K.stream_wait(torch.cuda.current_stream(side.device), side)
        _JOINED[dev] = n
    torch.autograd.Variable._execution_engine.queue_callback(join)


def _conv3x3_bn_fp8(a1, w_param, act, training, bn_params, bufs, mom, eps, pro=None):
    """conv2 (3x3, stride 1) forward on the fp8 halo kernel: a1 quantised to e4m3 in the kernel's halo staging
    (delayed scaling, no separate quantisation pass), e4m3 weight (current scaling, once per weight version),
    fused BN statistics."""
    from .fp8 import weight_fp8
    wq, winv = weight_fp8(w_param, krsc=True)
    t, slab = K.conv3x3_fp8(a1, wq, winv, act, want_stats=training, pro=pro)
    M = t.numel() // t.shape[-1]
    if training:
        mean, inv, sc, sh = _bn_train(slab, M, bn_params, bufs, mom, eps)
    else:
        mean, inv, sc, sh = _bn_eval(bn_params, bufs, eps)
    return t, mean, inv, sc, sh


class Fp8Conv2:
    """fp8 state of one Bottleneck's 3x3 conv (BASELINE.json config 5): the forward operand a1 in e4m3, the data
    gradient's operand dt2 in e5m2, each with its own delayed scale."""

    def __init__(self, device):
        from .fp8 import Fp8Act
        self.fwd = Fp8Act(device)
        self.bwd = Fp8Act(device, e5m2=True)


def _shortcut_fwd(x, kd, stride, training, bn_params, bufs, mom, eps):
    """The projection shortcut conv + BN statistics -> ((td, mean, invstd, scale, shift), its input).  Stride 2
    (tuning ds_sub): the conv reads a contiguous copy of x's even pixels, so it runs as a stride-1 1x1 conv and its
    weight gradient as a plain GEMM (the implicit-GEMM engine's strided gathers ran the ResNet-50 shortcut forwards at
    7-10% and their weight gradients at 5-13% of the bf16 peak: 0.86 + 1.04 ms per step, r5_52 trace)."""
    if stride > 1 and tuning.get("ds_sub") and x.shape[-1] % 8 == 0:
        xs = K.subsample(x, stride)
        return _conv_bn(xs, kd, 1, 0, None, training, bn_params, bufs, mom, eps), xs
    return _conv_bn(x, kd, stride, 0, None, training, bn_params, bufs, mom, eps), x


def _bn_back(g2d, t2d, mean, inv, gamma, mode, msrc=None, msc=None, msh=None, sink=None, bn_params=None):
    slab, _, rows = K.bn_bwd_reduce(g2d, t2d, mean, inv, mode=mode, msrc=msrc, mscale=msc, mshift=msh)
    if sink is not None:
        (dgamma, dbeta), (rg, rb) = sink.bn(slab, rows, *bn_params)
        dt, _, _ = K.bn_bwd_apply(g2d, t2d, mean, inv, gamma, dgamma, dbeta, mode=mode, msrc=msrc, mscale=msc,
                                  mshift=msh)
        return dt, rg, rb
    dgamma, dbeta = K.bn_bwd_finalize(slab, rows)
    dt, _, _ = K.bn_bwd_apply(g2d, t2d, mean, inv, gamma, dgamma, dbeta, mode=mode, msrc=msrc, mscale=msc,
                              mshift=msh)
    return dt, dgamma, dbeta


def _dgrad_bn_gm(dy, wk, t, st, pad, mean, inv, sc, sh, sink, gamma_p, beta_p, wprep=None):
    """dgrad with the fused BN-backward epilogue, stopped before the apply pass: -> (gm, dgamma, dbeta,
    returned grads).  The apply then runs inside the next data gradient's operand loads (_dgrad_pre)."""
    gm, slab = K.conv_dgrad(dy, wk, t.shape, st, pad, bn=(t, mean, inv, sc, sh), wprep=wprep)
    (dgamma, dbeta), ret = sink.bn(slab, slab.shape[0] // 2, gamma_p, beta_p)
    return gm, dgamma, dbeta, ret


_FWD_FORKED = {}      # device index -> flat.SHADOW_EPOCH when the side stream last waited on the compute stream
                      # in this model forward (a later mid-forward shadow re-cast needs a new fork)
_WPREP_SEQ = [0]      # wprep events in issue order
_WPREP_WAITED = {}    # device index -> highest wprep sequence number the compute stream has waited on


@contextlib.contextmanager
def side_forward(dev):
    """Around a model's block loop: the side stream waits on the compute stream ONCE (the optimizer step that
    refreshed the weights is then behind it), so the blocks' weight transforms need no fork of their own (one
    fork per block: 10,819-10,821 vs 10,844-10,853 img/s, gpurun_out/r3_73)."""
    side = _side_stream(dev) if dev.type == "cuda" else None
    if side is None:
        yield
        return
    K.stream_wait(side, torch.cuda.current_stream(dev))
    _FWD_FORKED[dev.index] = SHADOW_EPOCH[0]
    try:
        yield
    finally:
        _FWD_FORKED.pop(dev.index, None)


def _wait_wprep(dev, ev, seq):
    """The backward's wait for its block's transformed weights.  The side stream is in order, so waiting on the
    latest wprep event covers every earlier one: only the first block of the backward (the last of the forward)
    waits."""
    if _WPREP_WAITED.get(dev.index, -1) >= seq:
        return
    torch.cuda.current_stream(dev).wait_event(ev)
    _WPREP_WAITED[dev.index] = max(seq, _WPREP_WAITED.get(dev.index, -1))


def _prep_dgrad_weights(x, specs):
    """Make the data gradients' transformed weights (K.dgrad_weight: flipped 3x3, transposed 1x1) in the
    forward, on the side stream, which is idle there: the backward then finds them ready instead of running
    ~30 small transform kernels on its critical path.  specs: [(dy_shape, w, x_shape, st, pad)].
    -> (list of weights or None, event the backward waits on) or None without a side stream."""
    side = _side_stream(x.device)
    if side is None:
        return None
    main = torch.cuda.current_stream(x.device)
    idx = x.device.index
    if _FWD_FORKED.get(idx) != SHADOW_EPOCH[0]:
        # no fork in this forward yet, or a shadow slice was re-cast on the compute stream since the last one
        # (a PS weight bucket that landed mid-forward): the transforms must read the fresh weights
        K.stream_wait(side, main)
        if idx in _FWD_FORKED:
            _FWD_FORKED[idx] = SHADOW_EPOCH[0]
    with torch.cuda.stream(side):
        ws = [K.dgrad_weight(*sp) if sp is not None else None for sp in specs]
        ev = torch.cuda.Event()
        ev.record(side)
    for sp, w in zip(specs, ws):
        if sp is None:
            continue
        sp[1].record_stream(side)
        if w is not None:
            w.record_stream(main)
    _WPREP_SEQ[0] += 1
    return ws, (ev, _WPREP_SEQ[0])


def _pre_ok(t, wk, st, pad):
    """Whether the consumer of dt = bn_bwd_apply(gm, t) (data gradient of the conv with weight wk) takes the
    apply as its operand prologue."""
    return K.dgrad_pre_ok(tuple(t.shape), tuple(wk.shape), st, pad)


def _fused_dgrad_bn(dy, wk, t, st, pad, mean, inv, sc, sh, gamma, sink, gamma_p, beta_p, wprep=None):
    """dgrad whose epilogue applies the ReLU mask of relu(bn(t)) and reduces the BN-backward sums; then
    one apply pass produces dt (the gradient w.r.t. the BN input t)."""
    gm, slab = K.conv_dgrad(dy, wk, t.shape, st, pad, bn=(t, mean, inv, sc, sh), wprep=wprep)
    (dgamma, dbeta), ret = sink.bn(slab, slab.shape[0] // 2, gamma_p, beta_p)
    C = t.shape[-1]
    dt, _, _ = K.bn_bwd_apply(gm.view(-1, C), t.view(-1, C), mean, inv, gamma, dgamma, dbeta, mode=0)
    return dt.view(t.shape), ret[0], ret[1]


def _krsc_grad(dw):
    """fp32 [K][R][S][C] -> [K][C][R][S] view with channels_last strides (the parameter's layout)."""
    return dw.permute(0, 3, 1, 2)


class BottleneckFn(torch.autograd.Function):
    """Bottleneck (expansion 4): params = (w1,g1,b1, w2,g2,b2, w3,g3,b3[, wd,gd,bd])."""

    @staticmethod
    def forward(ctx, x, conf, bufs, shadows, *params):
        stride, training, mom, eps = conf[:4]
        fp8_meta = conf[4] if len(conf) > 4 else None
        down = len(params) == 12
        w1, g1, b1, w2, g2, b2, w3, g3, b3 = params[:9]
        k1, k2, k3 = shadows[:3]
        side_down = None
        xd = x                           # the shortcut conv's input (x, or its stride-2 subsample)
        side = _side_stream(x.device) if down else None
        if side is not None:
            # the shortcut conv only depends on x: run it (and its BN statistics) beside conv1 -> conv2 -> conv3
            main = torch.cuda.current_stream(x.device)
            K.stream_wait(side, main)
            with torch.cuda.stream(side):
                side_down, xd = _shortcut_fwd(x, shadows[3], stride, training, (params[10], params[11]), bufs[6:8],
                                              mom, eps)
            x.record_stream(side)
            for t in side_down + (xd,):
                t.record_stream(main)
        t1, m1, i1, s1, h1 = _conv_bn(x, k1, 1, 0, None, training, (g1, b1), bufs[0:2], mom, eps)
        C1 = t1.shape[-1]
        if stride == 1 and K.conv3x3_pro_ok(tuple(t1.shape), w2.shape[0]):
            # a1 = relu(bn1(t1)) is never materialised: the halo conv and the direct weight gradient apply BN1 + ReLU
            # while staging t1 (each element staged ~1.2x: one read of t1 instead of a bn_apply pass writing a1;
            # +0.2% ResNet-50 / +0.3% ResNet-152 same box, gpurun_out/r4_52)
            a1, pro1, src1 = None, (s1, h1), t1
        elif stride == 2 and K.conv3x3s2_a1_ok(tuple(t1.shape), w2.shape[0]) and not (
                fp8_meta is not None and K.conv3x3_fp8_ok(*t1.shape, w2.shape[0])):
            # stride 2 (tuning s2_halo bit 64): the half-resolution halo conv applies BN1 + ReLU while staging t1's
            # parity planes and writes the result as a1 for the weight gradient -- no separate bn_apply pass
            a1, pro1, src1 = torch.empty_like(t1), (s1, h1), t1
        elif stride == 2 and K.conv3x3s2_fold_ok(tuple(t1.shape), w2.shape[0]):
            # stride 2 (tuning s2_halo bit 4): the half-resolution halo conv applies BN1 + ReLU while staging each
            # parity plane of t1, the weight gradient through its operand prologue
            a1, pro1, src1 = None, (s1, h1), t1
        else:
            # the implicit-GEMM engine gathers every element 9 times: materialise a1 once instead
            a1 = K.bn_apply(t1.view(-1, C1), s1, h1, relu=True).view(t1.shape)
            pro1, src1 = None, a1
        fp8 = fp8_meta if (fp8_meta is not None and stride == 1
                           and K.conv3x3_fp8_ok(*t1.shape, w2.shape[0])) else None
        if fp8 is not None:
            t2, m2, i2, s2, h2 = _conv3x3_bn_fp8(src1, w2, fp8.fwd, training, (g2, b2), bufs[2:4], mom, eps, pro=pro1)
        elif a1 is not None and pro1 is not None:      # a1 written by the stride-2 forward (bit 64 above)
            t2, slab2 = K.conv3x3s2(t1, k2, want_stats=training, pro=pro1, pro_out=a1)
            if training:
                m2, i2, s2, h2 = _bn_train(slab2, t2.numel() // t2.shape[-1], (g2, b2), bufs[2:4], mom, eps)
            else:
                m2, i2, s2, h2 = _bn_eval((g2, b2), bufs[2:4], eps)
        else:
            t2, m2, i2, s2, h2 = _conv_bn(src1, k2, stride, 1, pro1, training, (g2, b2), bufs[2:4], mom, eps)
        # a2 = relu(bn2(t2)): on the A-stationary 1x1 kernel conv3 applies BN2 + ReLU to its activation fragments
        # once per pixel tile as they are loaded (and its weight gradient in the implicit-GEMM engine's operand
        # prologue), so a2 is never written (tuning a2_fold); elsewhere it is written once -- the 128-row engine's
        # prologue re-ran the affine for every 64-column output tile (gpurun_out/r3_03: 2.82 ms/step vs 0.29 +
        # 1.87 materialised)
        C2 = t2.shape[-1]
        fold = tuning.get("a2_fold")
        P2 = t2.numel() // C2
        if fold and K.conv1x1_pro_ok(tuple(t2.shape), k3.shape[0]) and (fold == 2 or P2 > K.WGRAD1X1_PP_PIX):
            a2, pro2, src2 = None, (s2, h2), t2
        else:
            a2 = K.bn_apply(t2.view(-1, C2), s2, h2, relu=True).view(t2.shape)
            pro2, src2 = None, a2
        t3, m3, i3, s3, h3 = _conv_bn(src2, k3, 1, 0, pro2, training, (g3, b3), bufs[4:6], mom, eps)
        C3 = t3.shape[-1]
        if down:
            if side_down is not None:
                K.stream_wait(main, side)
                td, md, idd, sd, hd = side_down
            else:
                (td, md, idd, sd, hd), xd = _shortcut_fwd(x, shadows[3], stride, training, (params[10], params[11]),
                                                          bufs[6:8], mom, eps)
            out, mb = K.bn_apply(t3.view(-1, C3), s3, h3, res=td.view(-1, C3), rscale=sd, rshift=hd, relu=True,
                                 want_mask=training)
        else:
            td = md = idd = None
            out, mb = K.bn_apply(t3.view(-1, C3), s3, h3, res=x.view(-1, C3), relu=True, want_mask=training)
        out = out.view(t3.shape)
        ctx.wprep = None
        if training:
            # (an fp8 conv2 takes its flipped e4m3 weight from ops.fp8.weight_fp8_flip instead)
            ctx.wprep = _prep_dgrad_weights(x, [(tuple(t3.shape), k3, tuple(t2.shape), 1, 0),
                                                (tuple(t2.shape), k2, tuple(t1.shape), stride, 1) if fp8 is None
                                                else None,
                                                (tuple(t1.shape), k1, tuple(x.shape), 1, 0)])
        # backward needs only the ReLU mask of `out`: 1 bit per element (mask mode 3), not the bf16 tensor
        ctx.save_for_backward(x, t1, a1, t2, t3, td, mb, m1, i1, s1, h1, m2, i2, s2, h2, m3, i3, md, idd,
                              g1, g2, g3, params[10] if down else None, k1, k2, k3, shadows[3] if down else None, a2,
                              xd if (down and xd is not x) else None)
        ctx.conf = (stride, training, down)
        ctx.params = params
        ctx.fp8 = fp8
        return out

    @staticmethod
    def backward(ctx, gout):
        (x, t1, a1, t2, t3, td, mb, m1, i1, s1, h1, m2, i2, s2, h2, m3, i3, md, idd,
         g1, g2, g3, gd, k1, k2, k3, kd, a2, xs) = ctx.saved_tensors
        stride, training, down = ctx.conf
        if not training:
            raise RuntimeError("fused Bottleneck backward requires training-mode BatchNorm")
        gout = gout.contiguous()
        C3 = t3.shape[-1]
        g2d, t3_2d = gout.view(-1, C3), t3.view(-1, C3)
        # block output BN3 (+BNd) with the ReLU mask of `out`
        P = ctx.params
        ctx.params = None
        sink = _Sink(gout.device)
        w3p = w2p = w1p = None
        if ctx.wprep is not None:
            (w3p, w2p, w1p), (ev, seq) = ctx.wprep
            _wait_wprep(gout.device, ev, seq)
            ctx.wprep = None
        gres_mask = mb if MASKED_RES else None
        slab3, slabd, rows = K.bn_bwd_reduce(g2d, t3_2d, m3, i3, mode=3, msrc=mb,
                                             x2=td.view(-1, C3) if down else None, mean2=md, invstd2=idd)
        (dg3, db3), (rg3, rb3) = sink.bn(slab3, rows, P[7], P[8])
        if down:
            (dgd, dbd), (rgd, rbd) = sink.bn(slabd, rows, P[10], P[11])
            dt3, dtd, _ = K.bn_bwd_apply(g2d, t3_2d, m3, i3, g3, dg3, db3, mode=3, msrc=mb,
                                         x2=td.view(-1, C3), mean2=md, invstd2=idd, gamma2=gd, dgamma2=dgd,
                                         dbeta2=dbd)
            gres = None
        elif MASKED_RES:
            # the identity branch's gradient gout * mask is added by conv1's data gradient (res_mask), not
            # materialised here: one activation-sized write less per block
            dt3, _, _ = K.bn_bwd_apply(g2d, t3_2d, m3, i3, g3, dg3, db3, mode=3, msrc=mb)
            gres = gout
        else:
            dt3, _, gres = K.bn_bwd_apply(g2d, t3_2d, m3, i3, g3, dg3, db3, mode=3, msrc=mb, want_gm=True)
        dt3 = dt3.view(t3.shape)
        # conv3 (input a2 = relu(bn2(t2)), or t2 with BN2 + ReLU as the operand prologue when a2 was folded)
        dw3 = sink.wgrad(P[6], a2 if a2 is not None else t2, dt3, 1, 1, 1, 0, pro=None if a2 is not None else (s2, h2))
        bn1 = (t1, m1, i1, s1, h1)
        if _pre_ok(t2, k2, stride, 1):
            # BN2's apply runs in conv2's data-gradient operand loads, which also write dt2 for the wgrad
            gm2, dg2, db2, (rg2, rb2) = _dgrad_bn_gm(dt3, k3, t2, 1, 0, m2, i2, s2, h2, sink, P[4], P[5], wprep=w3p)
            dt2 = torch.empty_like(t2)
            pre2 = (t2, m2, i2, g2, dg2, db2, dt2)
            if ctx.fp8 is not None:
                # fp8 data gradient: dt2 (applied in the halo staging) quantised to e5m2 there, tap-flipped e4m3 weight
                from .fp8 import weight_fp8_flip
                wt8, winv = weight_fp8_flip(P[3])
                gm1, slab1 = K.conv3x3_fp8(gm2, wt8, winv, ctx.fp8.bwd, bn=bn1, pre=pre2)
            else:
                gm1, slab1 = K.conv_dgrad(gm2, k2, t1.shape, stride, 1, bn=bn1, pre=pre2, wprep=w2p)
            del gm2
            dw2 = sink.wgrad(P[3], a1 if a1 is not None else t1, dt2, 3, 3, stride, 1,
                             pro=None if a1 is not None else (s1, h1), fp8=ctx.fp8)
        else:
            dt2, rg2, rb2 = _fused_dgrad_bn(dt3, k3, t2, 1, 0, m2, i2, s2, h2, g2, sink, P[4], P[5], wprep=w3p)
            dw2 = sink.wgrad(P[3], a1 if a1 is not None else t1, dt2, 3, 3, stride, 1,
                             pro=None if a1 is not None else (s1, h1))
            gm1, slab1 = K.conv_dgrad(dt2, k2, t1.shape, stride, 1, bn=bn1, wprep=w2p)
        (dg1, db1), (rg1, rb1) = sink.bn(slab1, slab1.shape[0] // 2, P[1], P[2])
        pre1 = None
        if _pre_ok(t1, k1, 1, 0):
            dt1 = torch.empty_like(t1)
            pre1 = (t1, m1, i1, g1, dg1, db1, dt1)
            dy1 = gm1
        else:
            C1 = t1.shape[-1]
            dt1 = K.bn_bwd_apply(gm1.view(-1, C1), t1.view(-1, C1), m1, i1, g1, dg1, db1, mode=0)[0].view(t1.shape)
            dw1 = sink.wgrad(P[0], x, dt1, 1, 1, 1, 0)
            dy1 = dt1
        if down:
            dtd = dtd.view(td.shape)
            # (with the subsampled input the shortcut's weight gradient is a plain GEMM: dtd^T . xs)
            dwd = sink.wgrad(P[9], xs, dtd, 1, 1, 1, 0) if xs is not None else sink.wgrad(P[9], x, dtd, 1, 1, stride, 0)
            dx = K.conv_dgrad(dy1, k1, x.shape, 1, 0, pre=pre1, wprep=w1p)
            # shortcut branch accumulated in place: a stride-2 1x1 dgrad only touches the pixels its taps
            # reach, so no zero-filled full-size buffer and no extra full read/write pass
            dx = K.conv_dgrad(dtd, kd, x.shape, stride, 0, res=dx, out=dx)
        else:
            dx = K.conv_dgrad(dy1, k1, x.shape, 1, 0, res=gres.view(x.shape), res_mask=gres_mask, pre=pre1,
                              wprep=w1p)
        if pre1 is not None:
            dw1 = sink.wgrad(P[0], x, dt1, 1, 1, 1, 0)       # dt1 written by conv1's data gradient
        grads = (dw1, rg1, rb1, dw2, rg2, rb2, dw3, rg3, rb3) + ((dwd, rgd, rbd) if down else ())
        sink.done()
        return (dx, None, None, None) + grads


class BasicBlockFn(torch.autograd.Function):
    """BasicBlock (expansion 1): params = (w1,g1,b1, w2,g2,b2[, wd,gd,bd])."""

    @staticmethod
    def forward(ctx, x, conf, bufs, shadows, *params):
        stride, training, mom, eps = conf
        down = len(params) == 9
        w1, g1, b1, w2, g2, b2 = params[:6]
        k1, k2 = shadows[:2]
        t1, m1, i1, s1, h1 = _conv_bn(x, k1, stride, 1, None, training, (g1, b1), bufs[0:2], mom, eps)
        C1 = t1.shape[-1]
        a1 = K.bn_apply(t1.view(-1, C1), s1, h1, relu=True).view(t1.shape)    # 3x3 consumer: materialise
        t2, m2, i2, s2, h2 = _conv_bn(a1, k2, 1, 1, None, training, (g2, b2), bufs[2:4], mom, eps)
        C2 = t2.shape[-1]
        xd = x
        if down:
            wd, gd, bd = params[6:]
            (td, md, idd, sd, hd), xd = _shortcut_fwd(x, shadows[2], stride, training, (gd, bd), bufs[4:6], mom, eps)
            out, mb = K.bn_apply(t2.view(-1, C2), s2, h2, res=td.view(-1, C2), rscale=sd, rshift=hd, relu=True,
                                 want_mask=training)
        else:
            td = md = idd = None
            out, mb = K.bn_apply(t2.view(-1, C2), s2, h2, res=x.view(-1, C2), relu=True, want_mask=training)
        out = out.view(t2.shape)
        ctx.save_for_backward(x, t1, a1, t2, td, mb, m1, i1, s1, h1, m2, i2, md, idd, g1, g2,
                              params[7] if down else None, k1, k2, shadows[2] if down else None,
                              xd if xd is not x else None)
        ctx.conf = (stride, training, down)
        ctx.params = params
        return out

    @staticmethod
    def backward(ctx, gout):
        (x, t1, a1, t2, td, mb, m1, i1, s1, h1, m2, i2, md, idd, g1, g2, gd, k1, k2, kd, xs) = ctx.saved_tensors
        stride, training, down = ctx.conf
        if not training:
            raise RuntimeError("fused BasicBlock backward requires training-mode BatchNorm")
        gout = gout.contiguous()
        C2 = t2.shape[-1]
        g2d, t2_2d = gout.view(-1, C2), t2.view(-1, C2)
        P = ctx.params
        ctx.params = None
        sink = _Sink(gout.device)
        slab2, slabd, rows = K.bn_bwd_reduce(g2d, t2_2d, m2, i2, mode=3, msrc=mb,
                                             x2=td.view(-1, C2) if down else None, mean2=md, invstd2=idd)
        (dg2, db2), (rg2, rb2) = sink.bn(slab2, rows, P[4], P[5])
        if down:
            (dgd, dbd), (rgd, rbd) = sink.bn(slabd, rows, P[7], P[8])
            dt2, dtd, _ = K.bn_bwd_apply(g2d, t2_2d, m2, i2, g2, dg2, db2, mode=3, msrc=mb, x2=td.view(-1, C2),
                                         mean2=md, invstd2=idd, gamma2=gd, dgamma2=dgd, dbeta2=dbd)
            gres = None
        else:
            dt2, _, _ = K.bn_bwd_apply(g2d, t2_2d, m2, i2, g2, dg2, db2, mode=3, msrc=mb)
            gres = gout                                     # masked by conv1's data-gradient epilogue
        dt2 = dt2.view(t2.shape)
        dw2 = sink.wgrad(P[3], a1, dt2, 3, 3, 1, 1)
        if _pre_ok(t1, k1, stride, 1):
            # BN1's apply inside conv1's data-gradient operand loads (dt1 written there for the wgrad)
            gm1, dg1, db1, (rg1, rb1) = _dgrad_bn_gm(dt2, k2, t1, 1, 1, m1, i1, s1, h1, sink, P[1], P[2])
            dt1 = torch.empty_like(t1)
            pre1, dy1 = (t1, m1, i1, g1, dg1, db1, dt1), gm1
        else:
            dt1, rg1, rb1 = _fused_dgrad_bn(dt2, k2, t1, 1, 1, m1, i1, s1, h1, g1, sink, P[1], P[2])
            dw1 = sink.wgrad(P[0], x, dt1, 3, 3, stride, 1)
            pre1, dy1 = None, dt1
        if down:
            dtd = dtd.view(td.shape)
            dwd = sink.wgrad(P[6], xs, dtd, 1, 1, 1, 0) if xs is not None else sink.wgrad(P[6], x, dtd, 1, 1, stride, 0)
            dx = K.conv_dgrad(dy1, k1, x.shape, stride, 1, pre=pre1)
            dx = K.conv_dgrad(dtd, kd, x.shape, stride, 0, res=dx, out=dx)      # shortcut, in place
        else:
            dx = K.conv_dgrad(dy1, k1, x.shape, stride, 1, res=gres.view(x.shape), res_mask=mb, pre=pre1)
        if pre1 is not None:
            dw1 = sink.wgrad(P[0], x, dt1, 3, 3, stride, 1)
        grads = (dw1, rg1, rb1, dw2, rg2, rb2) + ((dwd, rgd, rbd) if down else ())
        sink.done()
        return (dx, None, None, None) + grads


class StemFn(torch.autograd.Function):
    """conv(k, stride, pad) -> BN -> ReLU [-> maxpool(3, 2, 1)] on a channel-padded NHWC input.

    params = (w, gamma, beta); the weight shadow is zero-padded to the input's channel count."""

    @staticmethod
    def forward(ctx, x, conf, bufs, shadows, w, gamma, beta):
        stride, pad, pool, training, mom, eps = conf
        kpad = shadows[0]
        nchw = kpad.dim() == 3          # shadow from K.stem_weight_nchw: x is the NCHW bf16 batch itself
        direct = nchw or (pool and K.stem_ok(x.shape, kpad.shape, stride, pad))
        xn = None
        if nchw:
            # the weight gradient reads the NCHW batch itself (stem_wgrad.hip): no NHWC copy at all
            t, slab = K.stem_conv_nchw(x, kpad, want_stats=training)
            xn = x
        if direct:
            # direct 7x7/s2 kernel, then BN + ReLU + max-pool in one pass over t; the backward recomputes the
            # ReLU mask from t (mask mode 2), so neither the activation nor its mask is stored
            if not nchw:
                t, slab = K.stem_conv(x, kpad, want_stats=training)
            M = t.numel() // t.shape[-1]
            if training:
                m, i, s, h = _bn_train(slab, M, (gamma, beta), bufs, mom, eps)
            else:
                m, i, s, h = _bn_eval((gamma, beta), bufs, eps)
            y, idx = K.bn_relu_maxpool(t, s, h)
            mb = None
        else:
            t, m, i, s, h = _conv_bn(x, kpad, stride, pad, None, training, (gamma, beta), bufs, mom, eps)
            C = t.shape[-1]
            a, mb = K.bn_apply(t.view(-1, C), s, h, relu=True, want_mask=training)
            a = a.view(t.shape)
            if pool:
                y, idx = K.maxpool_fwd(a, 3, 2, 1)
            else:
                y, idx = a, None
        ctx.save_for_backward(x, t, mb, idx, m, i, gamma, s if direct else None, h if direct else None)
        ctx.nchw_wgrad = xn is not None
        ctx.conf = (stride, pad, pool, w.shape, (w.shape[0], 7, 7, 8) if nchw else kpad.shape)
        ctx.params = (w, gamma, beta)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, t, mb, idx, m, i, gamma, s, h = ctx.saved_tensors
        stride, pad, pool, wshape, kshape = ctx.conf
        gy = gy.contiguous()
        C = t.shape[-1]
        P = ctx.params
        ctx.params = None
        sink = _Sink()
        if ctx.nchw_wgrad and mb is None:
            # the BN backward's apply runs inside the NCHW weight-gradient kernel's staging: dt never written;
            # its statistics come out of the max-pool gather's pass
            fused = K.maxpool_bwd_bnred(gy, idx, t, m, i, s, h) if pool else None
            if fused is not None:
                ga, slab, rows = fused
            else:
                ga = K.maxpool_bwd(gy, idx, t.shape, 3, 2, 1) if pool else gy
                slab, _, rows = K.bn_bwd_reduce(ga.view(-1, C), t.view(-1, C), m, i, mode=2, msrc=t.view(-1, C),
                                               mscale=s, mshift=h)
            (dg_, db_), (dg, db) = sink.bn(slab, rows, P[1], P[2])
            pre = (t, m, i, gamma, dg_, db_, s, h)
            acc = sink.acc(P[0])
            if acc is not None and acc[0].stride() == (147, 1, 21, 3):
                K.stem_wgrad_nchw(x, ga, pre=pre, acc=acc[0])       # added straight into the arena
                dw = None
            else:
                dw = K.stem_wgrad_nchw(x, ga, pre=pre)
                if acc is not None:
                    acc[0].add_(dw)
                    dw = None
            sink.done()
            return None, None, None, None, dw, dg, db
        ga = K.maxpool_bwd(gy, idx, t.shape, 3, 2, 1) if pool else gy
        if mb is None:          # direct stem: ReLU mask recomputed from t (t * s + h > 0)
            dt, dg, db = _bn_back(ga.view(-1, C), t.view(-1, C), m, i, gamma, 2, msrc=t.view(-1, C), msc=s, msh=h,
                                  sink=sink, bn_params=(P[1], P[2]))
        else:
            dt, dg, db = _bn_back(ga.view(-1, C), t.view(-1, C), m, i, gamma, 3, msrc=mb, sink=sink,
                                  bn_params=(P[1], P[2]))
        dt = dt.view(t.shape)
        if kshape[3] == wshape[1]:
            dw = sink.wgrad(P[0], x, dt, kshape[1], kshape[2], stride, pad)
        else:
            dwk = K.conv_wgrad(x, dt, kshape[1], kshape[2], stride, pad)     # [K][R][S][Cpad]
            dw = dwk[:, :, :, : wshape[1]].permute(0, 3, 1, 2)
        sink.done()
        # the stem input is the data batch: no input gradient is produced
        return None, None, None, None, dw, dg, db


def stem_shadow(w, cpad):
    """bf16 [K][R][S][Cpad] weight for a channel-padded stem input."""
    k = weight_bf16(w, krsc=True)
    if k.shape[-1] != cpad:
        k = torch.nn.functional.pad(k, (0, cpad - k.shape[-1])).contiguous()
    return k
