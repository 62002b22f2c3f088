"""FP8 (OCP e4m3) forward GEMMs with per-tensor delayed scaling (SURVEY.md §2.8 K-18 "fp8 MFMA GEMM with
per-tensor scaling"; BASELINE.json config 5 "ResNet-152 fp8 weights").

Recipe (the usual fp8-training split): forward GEMMs read fp8 operands on the block-scaled
``v_mfma_scale_f32_16x16x128_f8f6f4`` path (2x the bf16 MFMA rate; ``pdnn_gemm_fp8`` runs the ping-pong
engine with 128-byte fp8 slices, ``csrc/kernels/gemm_pp.hip`` DT = 1); backward GEMMs stay bf16 on the saved bf16 activations and the bf16 weight shadow.

* **Weights** are quantised with *current* scaling once per optimizer step (amax pass -> scale -> quant,
  three tiny launches), cached against the parameter's version counter like the bf16 shadow.
* **Activations** use *delayed* scaling: the quantisation kernel records the tensor's amax (one partial
  per block, no same-address atomics) while it converts with the scale derived from the previous step's
  amax; one small kernel then reduces the partials, forms the GEMM's dequantisation factor (1 / (s_x s_w))
  and rolls the scale forward.  No host synchronisation.
  The very first call primes the scale with a real amax pass.
"""
from __future__ import annotations

import torch

from . import kernels as K
from .functional import weight_bf16

F32 = torch.float32


class Fp8Meta:
    """Device-side scaling state of one fp8 GEMM input."""

    AMAX_PARTS = 1024      # per-block partial maxima written by quant_fp8 (csrc/kernels/fp8.hip FP8_AMAX_PARTS)

    def __init__(self, device, margin: int = 0):
        self.amax = torch.zeros(self.AMAX_PARTS, device=device, dtype=F32)
        self.scale = torch.ones(1, device=device, dtype=F32)
        self.inv = torch.ones(1, device=device, dtype=F32)
        self.gemm_scale = torch.ones(1, device=device, dtype=F32)
        self.margin = margin
        self.primed = False

    def quantize(self, x, inv_w):
        """-> (e4m3 bytes of x, device scalar 1 / (s_x * s_w) for the GEMM epilogue)."""
        if not self.primed:
            K.amax_(x, self.amax)
            K.fp8_scale(self.amax, self.scale, self.inv, self.margin)
            self.amax.zero_()
            self.primed = True
        q = K.quant_fp8(x, self.scale, amax=self.amax)
        K.fp8_scale_step(self.amax, self.scale, self.inv, inv_w, self.gemm_scale, self.margin)
        return q, self.gemm_scale


class Fp8Act:
    """Delayed-scaling state of an operand that a kernel quantises in-line (the fp8 halo conv: ``K.conv3x3_fp8``):
    the kernel reads ``scale``, records its staged |max| into the ``amax`` partials, and ``K.fp8_scale_roll``
    rolls the scale forward after it.  e5m2 for gradients (range), e4m3 for activations (precision)."""

    def __init__(self, device, e5m2: bool = False, margin: int = 0):
        self.amax = torch.zeros(Fp8Meta.AMAX_PARTS, device=device, dtype=F32)
        self.scale = torch.ones(1, device=device, dtype=F32)
        self.inv = torch.ones(1, device=device, dtype=F32)
        self.e5m2 = bool(e5m2)
        self.margin = margin
        self.primed = False


def _wait_prefetch(p):
    # made on the side stream by prefetch_fp8_weights: the compute stream waits once per prefetch (shared token)
    tok = p.__dict__.get("_pdnn_fp8_wait")
    if tok is not None:
        if not tok[1]:
            torch.cuda.current_stream(p.device).wait_event(tok[0])
            tok[1] = True
        p._pdnn_fp8_wait = None


def prefetch_fp8_weights(ps, side):
    """Make the e4m3 weights (and tap-flipped copies) of ``ps`` whose cache is stale on the ``side`` stream, at
    the start of a forward: ~17 us of small quantisation / flip kernels per 3x3 conv leave the compute stream
    (the first fp8 conv waits on one event).  Skipped for parameters still arriving (PS workers mark them
    ``_pdnn_weight_pending``; a k-of-n DDP forward check, which also hooks ``_pdnn_await``, does not)."""
    todo = [p for p in ps if "_pdnn_weight_pending" not in p.__dict__
            and (getattr(p, "_pdnn_fp8_flip", None) or (None,))[0] != _weight_version(p)]
    if not todo:
        return
    dev = todo[0].device
    main = torch.cuda.current_stream(dev)
    for p in todo:
        weight_bf16(p, krsc=True)          # the shadows current on the compute stream first
    K.stream_wait(side, main)
    with torch.cuda.stream(side):
        for p in todo:
            weight_fp8_flip(p)
        ev = torch.cuda.Event()
        ev.record(side)
    tok = [ev, False]
    for p in todo:
        p._pdnn_fp8_wait = tok
        p._pdnn_fp8[1].record_stream(main)
        p._pdnn_fp8[2].record_stream(main)
        p._pdnn_fp8_flip[1].record_stream(main)


def weight_fp8_flip(p: torch.Tensor):
    """(e4m3 tap-flipped transposed 3x3 weight [C][3][3][K], inverse scale) for the fp8 data gradient, made from
    weight_fp8's bytes (same scale) and cached per parameter version alongside it."""
    wq, inv = weight_fp8(p, krsc=True)
    _wait_prefetch(p)
    st = getattr(p, "_pdnn_fp8_flip", None)
    ver = _weight_version(p)
    if st is not None and st[0] == ver:
        return st[1], inv
    Kc, C = p.shape[0], p.shape[1]
    wt = K.conv3x3_flip8(wq, Kc, C)
    p._pdnn_fp8_flip = (ver, wt)
    return wt, inv


def _weight_version(p):
    # flat-arena parameters are updated in place by the fused optimizer (no autograd version bump):
    # key on the arena's update generation as well
    fp = getattr(p, "_pdnn_flat", None)
    return (p._version, fp.generation if fp is not None else 0)


def weight_fp8(p: torch.Tensor, krsc: bool = False):
    """(e4m3 weight [N][K] (conv: [K][R*S*C]), device inverse scale) cached per parameter version.
    Current scaling (exact amax of this version) in two launches: per-block amax partials, then a quantiser
    that reduces them itself (no fill, no single-thread scale kernel)."""
    from ..optim.flat import await_param
    await_param(p)                     # before the cache check: a PS bucket landing bumps the generation
    _wait_prefetch(p)
    st = getattr(p, "_pdnn_fp8", None)
    ver = _weight_version(p)
    if st is not None and st[0] == ver:
        return st[1], st[2]
    wb = weight_bf16(p, krsc=krsc)
    w2 = wb.reshape(wb.shape[0], -1).contiguous()
    inv = st[2] if st is not None else torch.empty(1, device=p.device, dtype=F32)
    q = K.quant_fp8_current(w2, inv, out=st[1] if st is not None and st[1].shape == w2.shape else None)
    p._pdnn_fp8 = (ver, q, inv)
    return q, inv


def fp8_ok(M, N, Kd):
    return Kd % 128 == 0 and N % 8 == 0 and M >= 1


def linear_fp8_fwd(x2, p_w, meta: Fp8Meta, bias=None, act=0, aux=None, res=None, stats=None):
    """y = act(x2 @ W^T + bias) (+res) with x2 and W in e4m3 (bf16 output) on the in-tree block-scaled
    MFMA engine (``pdnn_gemm_fp8``), optional fused BN statistics of the output."""
    wq, winv = weight_fp8(p_w)
    xq, gs = meta.quantize(x2, winv)
    return K.gemm_fp8(xq, wq, gs, bias=bias, act=act, aux=aux, res=res, stats=stats)
