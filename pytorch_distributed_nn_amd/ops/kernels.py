"""Typed Python wrappers around the HIP launchers (one function per kernel entry point).

Every wrapper checks the shape / dtype / layout contract the kernel assumes *on the host* before
launching (a bad launch can take down the whole GPU box), allocates outputs with torch's caching
allocator, and launches on torch's current stream.  Activations are NHWC bf16 tensors of shape
(N, H, W, C); conv weights are bf16 tensors whose memory is [K][R][S][C] (torch ``channels_last``).
"""
from __future__ import annotations

import ctypes

import torch

from ._backend import _CUR_DEV, call, lib, ptr, stream

BF16 = torch.bfloat16
F32 = torch.float32


def _chk(cond, msg):
    if not cond:
        raise ValueError(msg)


def _is_krsc(w):
    K, C, R, S = w.shape
    return w.stride() == (R * S * C, 1, S * C, C)


def _bf16_c(t, name):
    _chk(t.dtype == BF16 and t.is_cuda, f"{name}: expected CUDA bf16, got {t.dtype} {t.device}")
    _chk(t.is_contiguous(), f"{name}: expected contiguous tensor")
    _chk(t.data_ptr() % 16 == 0, f"{name}: 16-byte alignment required")


# ----------------------------------------------------------------------------------- GEMM / conv
def set_staged_store(mode: int) -> int:
    """128-row kernel bf16 epilogue: 1 = stores staged through LDS (full rows), 0 = direct fragment stores."""
    return lib().pdnn_set_staged_store(int(mode))


def set_glds_mode(mode: int) -> int:
    """GEMM engine selection: 1 automatic (default), 0 register-staged 128-tile kernel only, 2 the glds
    256-row engine whenever the operands allow it.  Returns the previous mode."""
    return lib().pdnn_set_glds_mode(int(mode))


def set_pp_mode(mode: int) -> int:
    """Ping-pong GEMM engine (csrc/kernels/gemm_pp.h) for plain GEMMs: 1 automatic (default), 0 off, 2 whenever
    the operands allow it.  Returns the previous mode."""
    return lib().pdnn_set_pp_mode(int(mode))


def set_pp_bn(bn: int) -> int:
    """Force the ping-pong engine's tile width (96/128/192/256/288; 0 = automatic).  Returns the previous."""
    return lib().pdnn_set_pp_bn(int(bn))


def pp_wgrad(x, y, out, alpha=1.0, splits=None, ws=None, rowsum=None, bn=0, plan_cus=0):
    """out[M][N] (fp32) += alpha * x[K][M]^T @ y[K][N] on the ping-pong engine: split-K partial slabs in a
    workspace (``ws``, allocated when not given) reduced by a second kernel, or in place when one split
    covers the CUs.  ``rowsum`` (fp32 [M], optional) += alpha * x.sum(0), fused: the bias gradient of a
    linear layer beside its weight gradient.  ``splits=None``: tile width and splits from the joint plan
    (pdnn_pp_wgrad_plan, for ``plan_cus`` CUs when > 0: a weight gradient beside other work on a side stream);
    ``bn`` (128 / 256, 0 = the engine's pick) only with explicit ``splits``."""
    K_, M = x.shape
    K2, N = y.shape
    _chk(K_ == K2 and K_ % 32 == 0 and M % 8 == 0 and N % 8 == 0, f"pp_wgrad: bad shapes {x.shape} {y.shape}")
    _chk(out.dtype == F32 and out.shape == (M, N) and out.stride(1) == 1, "pp_wgrad: fp32 [M][N] output")
    if splits is None:
        bn, splits = divmod(lib().pdnn_pp_wgrad_plan(M, N, K_, int(plan_cus)), 1000)
    if splits > 1 and ws is None:
        ws = torch.empty(splits * (M * N + 64), device=x.device, dtype=F32)     # pdnn_pp_wgrad_ws
    _chk(splits <= 1 or ws.numel() >= splits * (M * N + 64), "pp_wgrad: workspace of splits * (M*N + 64) floats")
    _chk(rowsum is None or (rowsum.dtype == F32 and rowsum.is_contiguous() and rowsum.numel() == M),
         "pp_wgrad: rowsum fp32 [M]")
    call("pdnn_pp_wgrad", ptr(x), x.stride(0), ptr(y), y.stride(0), ptr(out), out.stride(0), M, N, K_,
         float(alpha), ptr(ws), int(splits), ptr(rowsum), int(bn), stream())
    return out


def gemm_nt_splitk(x, w, splits=None, ws=None):
    """y[M][N] (bf16) = x[M][K] @ w[N][K]^T with the reduction split over work items writing fp32 slabs
    (for K >> M, N: e.g. the tied LM head's data gradient, K = vocabulary)."""
    M, Kd = x.shape
    N = w.shape[0]
    _chk(w.shape[1] == Kd and Kd % 32 == 0 and N % 8 == 0, f"gemm_nt_splitk: bad shapes {x.shape} {w.shape}")
    _chk(x.stride(1) == 1 and w.stride(1) == 1, "gemm_nt_splitk: K-contiguous operands")
    if splits is None:
        splits = lib().pdnn_pp_splitk_splits(M, N, Kd)
    if ws is None:
        ws = torch.empty(splits * (M * N + 64), device=x.device, dtype=F32)
    _chk(ws.numel() >= splits * (M * N + 64), "gemm_nt_splitk: workspace of splits * (M*N + 64) floats")
    out = torch.empty(M, N, device=x.device, dtype=BF16)
    call("pdnn_pp_gemm_nt_splitk", ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0), M, N, Kd,
         ptr(ws), int(splits), stream())
    return out


def subsample(x, st=2):
    """x[:, ::st, ::st, :] of an NHWC bf16 tensor, contiguous (the input a 1x1 / stride-st conv reads)."""
    _bf16_c(x, "subsample.x")
    N, H, W, C = x.shape
    _chk(C % 8 == 0, "subsample: C % 8 == 0")
    y = torch.empty(N, (H - 1) // st + 1, (W - 1) // st + 1, C, device=x.device, dtype=BF16)
    call("pdnn_subsample", ptr(x), ptr(y), N, H, W, C, int(st), stream())
    return y


def transpose_bf16(x, out=None):
    """out[C][R] = x[R][C] (bf16, 2-D, unit column stride)."""
    _chk(x.dtype == BF16 and x.dim() == 2 and x.stride(1) == 1, "transpose_bf16: 2-D bf16 with unit column stride")
    R, C = x.shape
    if out is None:
        out = torch.empty(C, R, device=x.device, dtype=BF16)
    call("pdnn_transpose_bf16", ptr(x), x.stride(0), ptr(out), out.stride(0), R, C, stream())
    return out


def transpose_bf16_multi(pairs):
    """dst[C][R] = src[R][C] for every (src, dst) of ``pairs`` (contiguous bf16 2-D), in one launch per 64."""
    n = len(pairs)
    if n == 0:
        return
    for s_, d_ in pairs:
        _chk(s_.dtype == BF16 and d_.dtype == BF16 and s_.dim() == 2 and s_.is_contiguous() and d_.is_contiguous()
             and d_.shape == (s_.shape[1], s_.shape[0]), "transpose_bf16_multi: contiguous bf16 [R][C] -> [C][R]")
    srcs = (ctypes.c_void_p * n)(*[s_.data_ptr() for s_, _ in pairs])
    dsts = (ctypes.c_void_p * n)(*[d_.data_ptr() for _, d_ in pairs])
    rs = (ctypes.c_int * n)(*[s_.shape[0] for s_, _ in pairs])
    cs = (ctypes.c_int * n)(*[s_.shape[1] for s_, _ in pairs])
    call("pdnn_transpose_bf16_multi", srcs, dsts, rs, cs, n, stream())


def gemm_nt(x, w, bias=None, relu=False, out_f32=False, alpha=1.0, out=None):
    """y[M][N] = alpha * x[M][K] @ w[N][K]^T (+bias)(relu).  x, w bf16 row-major."""
    M, K = x.shape
    N, K2 = w.shape
    _chk(K == K2 and K % 8 == 0, f"gemm_nt: K mismatch/alignment {x.shape} {w.shape}")
    _chk(x.stride(1) == 1 and w.stride(1) == 1 and x.stride(0) % 8 == 0 and w.stride(0) % 8 == 0,
         "gemm_nt: rows must be K-contiguous, 16B aligned")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=F32 if out_f32 else BF16)
    _chk(N % 8 == 0 or out_f32, "gemm_nt: N % 8 for bf16 output")
    call("pdnn_gemm_nt", ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0), M, N, K,
         float(alpha), ptr(bias), int(relu), int(out_f32), stream())
    return out


def gemm_nn(x, w, out_f32=False, alpha=1.0, out=None):
    """y[M][N] = alpha * x[M][K] @ w[K][N]."""
    M, K = x.shape
    K2, N = w.shape
    _chk(K == K2 and N % 8 == 0 and K % 8 == 0, f"gemm_nn: bad shapes {x.shape} {w.shape}")
    _chk(x.stride(1) == 1 and w.stride(1) == 1, "gemm_nn: row-major operands")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=F32 if out_f32 else BF16)
    call("pdnn_gemm_nn", ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0), M, N, K,
         float(alpha), int(out_f32), stream())
    return out


def gemm_tn_acc(x, y, out, alpha=1.0):
    """out[M][N] (fp32) += alpha * x[K][M]^T @ y[K][N]."""
    K, M = x.shape
    K2, N = y.shape
    _chk(K == K2 and M % 8 == 0 and N % 8 == 0, f"gemm_tn: bad shapes {x.shape} {y.shape}")
    _chk(out.dtype == F32 and out.shape == (M, N) and out.stride(1) == 1, "gemm_tn: fp32 [M][N] output")
    call("pdnn_gemm_tn_acc", ptr(x), x.stride(0), ptr(y), y.stride(0), ptr(out), out.stride(0), M, N, K,
         float(alpha), stream())
    return out


def conv_out_hw(H, W, R, S, st, pad):
    return (H + 2 * pad - R) // st + 1, (W + 2 * pad - S) // st + 1


def stats_rows(M: int) -> int:
    """Row pairs of a BatchNorm statistics slab (every producer adds into STAT_BINS bins)."""
    return STAT_BINS


# 3x3 / stride-1 / pad-1 convs run on the LDS-halo kernel (csrc/kernels/conv3x3.hip): 1 = whenever the
# shape is supported (default), 0 = the implicit-GEMM engine (tuning conv3x3 / set_conv3x3_mode)
from .. import tuning as _tuning
_C3 = {"mode": 1, "nb": 0}


def tune_set(key: str, value: int) -> int:
    """Set a kernel-side dispatch-table entry (csrc/kernels/tuning.h); returns the previous value."""
    old = lib().pdnn_tune_set(key.encode(), int(value))
    _chk(old != -2 ** 31, f"unknown kernel tuning key {key!r}")
    return old


def tune_get(key: str) -> int:
    v = lib().pdnn_tune_get(key.encode())
    _chk(v != -2 ** 31, f"unknown kernel tuning key {key!r}")
    return v


def set_comm_world(world: int) -> int:
    """Tell the kernels how many ranks this process's collectives span: above 1, the persistent grids leave
    ``tune_get("comm_cus")`` CUs to RCCL's channel blocks (csrc/kernels/tuning.h).  Returns the previous value."""
    return lib().pdnn_set_comm_world(int(world))


def grid_cus() -> int:
    """CUs a persistent grid fills under the current comm world and dispatch table."""
    return lib().pdnn_grid_cus()


def tune_table():
    """[(key, value, default, doc)] of the kernel-side dispatch table."""
    import ctypes
    n = lib().pdnn_tune_list(None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib().pdnn_tune_list(buf, n + 1)
    out = []
    for line in buf.value.decode().splitlines():
        kv, dflt, doc = line.split("|", 2)
        k, v = kv.split("=")
        out.append((k, int(v), int(dflt), doc))
    return out


def set_conv3x3_mode(mode: int, nb: int = 0):
    """Returns the previous (mode, nb).  nb: 0 automatic, 64 / 128 forced output-channel tile."""
    old = (_C3["mode"], _C3["nb"])
    _C3["mode"], _C3["nb"] = int(mode), int(nb)
    return old


def _conv3x3_ok(N, H, W, Cin, Cout, R, S, st, pad):
    return (_C3["mode"] and R == 3 and S == 3 and st == 1 and pad == 1
            and lib().pdnn_conv3x3_supported(N, H, W, Cin, Cout) == 1)


def _s2_ok(N, H, W, C, K, R, S, st, pad, bit):
    """3x3 / stride-2 / pad-1 conv of an H x W x C input with K outputs on the half-resolution halo kernels
    (csrc/kernels/conv_s2.hip) for this direction (tuning s2_halo bit: 1 data gradient, 2 forward, 16 the data
    gradient's BN-backward operand prologue).  The forward goes there only while its grid fills the chip at least
    twice (>= 512 blocks of 256 pixels x 128 channels): ResNet-50 stage 2 111 vs 139 us on the implicit-GEMM engine,
    stages 3 / 4 (392 / 196 blocks) 102 / 152 vs 91 / 101 (tools/bench_conv_s2.py, gpurun_out/r6_02); bit 32 forces
    it (tests)."""
    tb = _tuning.get("s2_halo")
    if not (R == 3 and S == 3 and st == 2 and pad == 1 and (tb & bit) != 0):
        return False
    if bit == 2 and not (tb & 32) and -(-N * (H // 2) * (W // 2) // 256) * (K // 128) < 512:
        return False
    return lib().pdnn_conv3x3s2_supported(N, H, W, C, K) == 1


def conv3x3s2_fold_ok(x_shape, Ko):
    """Whether a 3x3 / stride-2 conv of this input takes its input's BN + ReLU as the forward kernel's operand
    prologue (tuning s2_halo bit 4): its activation need not be materialised."""
    N, H, W, C = x_shape
    return (_tuning.get("s2_halo") & 4) != 0 and _s2_ok(N, H, W, C, Ko, 3, 3, 2, 1, 2) and (
        (_tuning.get("s2_halo") & 8) == 0 or lib().pdnn_conv3x3s2_wgrad_supported(N, H, W, C, Ko) == 1)


def conv3x3s2_a1_ok(x_shape, Ko):
    """Whether the stride-2 forward runs on the halo kernel here with its input's BN + ReLU applied while staging AND
    written out as a by-product (tuning s2_halo bit 64): the activation a1 is materialised for the weight gradient
    without a bn_apply pass."""
    N, H, W, C = x_shape
    return (_tuning.get("s2_halo") & 64) != 0 and _s2_ok(N, H, W, C, Ko, 3, 3, 2, 1, 2)


def conv3x3s2(x, w, dgrad=False, want_stats=False, bn=None, pre=None, pro=None, pro_out=None):
    """Stride-2 3x3 conv on the halo kernels.  Forward: y (N, H/2, W/2, K) = conv(x (N, H, W, C), w [K][3][3][C]),
    BN statistics bins (want_stats) and the forward prologue pro = (scale, shift).  Data gradient (dgrad=True):
    x = dy (N, Ho, Wo, K), w = conv3x3_flip(W) [C][3][3][K] -> dx (N, 2Ho, 2Wo, C) with the fused BN backward
    (bn, as conv_dgrad) and the BN-backward operand prologue (pre, _pre_args)."""
    Nimg, H, W, C = x.shape
    N = w.shape[0]
    if dgrad:
        Ho, Wo = H * 2, W * 2
    else:
        Ho, Wo = H // 2, W // 2
    y = torch.empty(Nimg, Ho, Wo, N, device=x.device, dtype=BF16)
    slab = None
    t = mean = inv = msc = msh = None
    if want_stats or bn is not None:
        slab = stat_bins(N, x.device)
    if bn is not None:
        t, mean, inv, msc, msh = bn
        _chk(tuple(t.shape) == (Nimg, Ho, Wo, N), "conv3x3s2: bn_x shape")
    psc, psh = pro if pro is not None else (None, None)
    pargs = _pre_args(pre, x)
    if pro_out is not None:         # forward: the prologue's output (a1) written as a by-product
        _chk(not dgrad and pro is not None and pre is None and pro_out.shape == x.shape and pro_out.dtype == BF16
             and pro_out.is_contiguous(), "conv3x3s2: pro_out needs the forward prologue and x's shape")
        pargs = (None,) * 6 + (ptr(pro_out),)
    pair = int(dgrad and pre is None and (_tuning.get("s2_halo") & 128) != 0)
    call("pdnn_conv3x3s2", ptr(x), ptr(w), ptr(y), Nimg, Ho if dgrad else H, Wo if dgrad else W, C, N, int(dgrad),
         ptr(slab), ptr(t), ptr(mean), ptr(inv), ptr(msc), ptr(msh), *pargs, ptr(psc), ptr(psh), pair, stream())
    return y, slab


# 1x1 / stride-1 convs with K in {64, 128, 256} run on the A-stationary kernel (csrc/kernels/conv3x3.hip), K >= 512
# on the long-reduction one (conv1x1_wide.hip): set_panel_mode(0) sends them back to the implicit-GEMM engines
_P1 = {"mode": 1}


def set_panel_mode(mode: int) -> int:
    old = _P1["mode"]
    _P1["mode"] = int(mode)
    return old


def _wide_ok(P, K, N, fwd):
    """1x1 / stride-1 data gradients with a long reduction and a wide output (K >= 512, N >= 1024: ResNet-50's
    stage-4 conv1 data gradients) on the streaming kernel (conv1x1_wide.hip; tuning wide1x1_dgrad): 81 vs 102 us
    on the ping-pong engine.  Not the forwards or the conv3 data gradients (N <= 512), where the implicit-GEMM
    engine stays ahead (gpurun_out/r4_02)."""
    return (not fwd and K >= 512 and N >= 1024 and _tuning.get("wide1x1_dgrad") == 1
            and lib().pdnn_conv1x1_wide_supported(P, K, N) == 1)


def _panel_ok(P, K, N, R, S, st, pad, fwd=False):
    return (_P1["mode"] and R == 1 and S == 1 and st == 1 and pad == 0
            and (lib().pdnn_conv1x1_panel_supported(P, K, N) == 1 or _wide_ok(P, K, N, fwd)))


def _pre_args(pre, x):
    """pre = (t, mean, invstd, gamma, dgamma, dbeta, dt_out or None): the BN-backward apply of the layer whose
    gradient gm is ``x`` (dt = bn_bwd_apply(gm, t), mode 0) fused into the operand loads."""
    if pre is None:
        return (None,) * 7
    t, mean, inv, gamma, dg, db, dt_out = pre
    _bf16_c(t, "pre.t")
    _chk(t.numel() == x.numel(), "pre: t must have the operand's shape")
    if dt_out is not None:
        _chk(dt_out.numel() == x.numel() and dt_out.dtype == BF16 and dt_out.is_contiguous(), "pre: dt_out")
    return tuple(ptr(v) for v in (t, mean, inv, gamma, dg, db, dt_out))


def conv1x1_panel(x2d, w2d, want_stats=False, res=None, bn=None, res_mask=None, out=None, pre=None, pro=None):
    """y[P][N] = x[P][K] . w[N][K]^T on the panel / A-stationary kernels (K <= 256) or the long-reduction kernel
    (K >= 512); epilogues as conv3x3 / conv_dgrad; pre: the BN-backward operand prologue (_pre_args); pro =
    (scale, shift): the forward operand prologue relu(x * scale + shift) (A-stationary kernel, K <= 256)."""
    P, Kc = x2d.shape
    N = w2d.shape[0]
    y = out if out is not None else torch.empty(P, N, device=x2d.device, dtype=BF16)
    slab = None
    t = mean = inv = msc = msh = None
    if want_stats or bn is not None:
        slab = stat_bins(N, x2d.device)
    if bn is not None:
        t, mean, inv, msc, msh = bn
    if Kc >= 512:
        _chk(pro is None, "conv1x1_panel: the forward prologue needs K <= 256")
        call("pdnn_conv1x1_wide", ptr(x2d), ptr(w2d), ptr(y), P, Kc, N, ptr(slab), ptr(res), ptr(res_mask), ptr(t),
             ptr(mean), ptr(inv), ptr(msc), ptr(msh), *_pre_args(pre, x2d), stream())
        return y, slab
    psc, psh = pro if pro is not None else (None, None)
    call("pdnn_conv1x1_panel", ptr(x2d), ptr(w2d), ptr(y), P, Kc, N, ptr(slab), ptr(res), ptr(res_mask), ptr(t),
         ptr(mean), ptr(inv), ptr(msc), ptr(msh), *_pre_args(pre, x2d), ptr(psc), ptr(psh), stream())
    return y, slab


def conv3x3_flip(w):
    """W'[C][3][3][K] = W[K][2-r][2-s][C] (bf16): the data gradient's weight for the halo kernel."""
    K, R, S, C = w.shape
    wt = torch.empty(C, 3, 3, K, device=w.device, dtype=BF16)
    call("pdnn_conv3x3_flip", ptr(w), ptr(wt), K, C, stream())
    return wt


def conv3x3(x, w, want_stats=False, res=None, bn=None, out=None, res_mask=None, pre=None, pro=None):
    """y = conv3x3(x, w) (stride 1, pad 1) on the halo kernel, w: bf16 [N][3][3][C].  Epilogues as
    conv_fwd / conv_dgrad (stats slab, residual add, fused BN backward).  pro = (scale, shift) fp32 [C]: the operand
    is relu(x * scale + shift), applied while the halo is staged (x is the BN input; plain / stats epilogues)."""
    Nimg, H, W, C = x.shape
    Ko = w.shape[0]
    y = out if out is not None else torch.empty(Nimg, H, W, Ko, device=x.device, dtype=BF16)
    slab = None
    t = mean = inv = msc = msh = None
    if want_stats or bn is not None:
        slab = stat_bins(Ko, x.device)
    if bn is not None:
        t, mean, inv, msc, msh = bn
    psc, psh = pro if pro is not None else (None, None)
    call("pdnn_conv3x3", ptr(x), ptr(w), ptr(y), Nimg, H, W, C, Ko, ptr(slab), ptr(res), ptr(res_mask), ptr(t),
         ptr(mean), ptr(inv), ptr(msc), ptr(msh), _C3["nb"], *_pre_args(pre, x), ptr(psc), ptr(psh), stream())
    return y, slab


def conv_fwd(x, w, st, pad, pro=None, want_stats=False):
    """x: NHWC bf16 (N,H,W,C); w: bf16 [K][R][S][C] memory (shape K,C,R,S channels_last or K,R,S,C).
    pro: optional (scale, shift) fp32 [C] -> input transformed relu(x*scale+shift) on load.
    Returns (y NHWC bf16, stats slab or None)."""
    _bf16_c(x, "conv_fwd.x")
    N, H, W, C = x.shape
    _bf16_c(w, "conv_fwd.w")
    K, R, S, C2 = w.shape
    _chk(C2 == C, f"conv_fwd: weight {tuple(w.shape)} must be [K][R][S][C] with C={C}")
    _chk(C % 8 == 0 and K % 8 == 0, f"conv_fwd: channels must be multiples of 8 (C={C}, K={K})")
    Ho, Wo = conv_out_hw(H, W, R, S, st, pad)
    if _conv3x3_ok(N, H, W, C, K, R, S, st, pad):
        return conv3x3(x, w, want_stats=want_stats, pro=pro)
    if _s2_ok(N, H, W, C, K, R, S, st, pad, 2):
        return conv3x3s2(x, w, want_stats=want_stats, pro=pro)
    if (pro is None or C <= 256) and _panel_ok(N * H * W, C, K, R, S, st, pad, fwd=True):
        y, slab = conv1x1_panel(x.view(-1, C), w.view(K, C), want_stats=want_stats, pro=pro)
        return y.view(N, H, W, K), slab
    y = torch.empty(N, Ho, Wo, K, device=x.device, dtype=BF16)
    stats = None
    if want_stats:
        stats = stat_bins(K, x.device)
    sc, sh = pro if pro is not None else (None, None)
    call("pdnn_conv_fwd", ptr(x), ptr(w), ptr(y), N, H, W, C, K, R, S, st, pad, Ho, Wo, ptr(sc), ptr(sh),
         ptr(stats), stream())
    return y, stats


def _panel_dgrad_k(K):
    """Data gradients (dx[P][C] = dy[P][K] . W) on the A-stationary kernel (K in {64, 128, 256}) or the
    long-reduction streaming kernel (K >= 512, conv1x1_wide.hip)."""
    return K in (64, 128, 256) or K >= 512


def conv1x1_pro_ok(x_shape, Ko):
    """Whether a 1x1 / stride-1 conv of this input runs with its input's BN + ReLU as an operand prologue on the
    A-stationary kernel (forward; its weight gradient then takes the same prologue on the implicit-GEMM engine)."""
    N, H, W, C = x_shape
    return bool(_P1["mode"]) and C in (64, 128, 256) and lib().pdnn_conv1x1_panel_supported(N * H * W, C, Ko) == 1


def conv3x3_pro_ok(x_shape, Ko):
    """Whether a 3x3 / stride-1 conv of this input takes its input's BN + ReLU as an operand prologue in both its
    forward (halo kernel) and its weight gradient (direct kernel): the activation then need not be materialised."""
    N, H, W, C = x_shape
    return _conv3x3_ok(N, H, W, C, Ko, 3, 3, 1, 1) and lib().pdnn_conv3x3_wgrad_supported(N, H, W, C, Ko) == 1


def dgrad_pre_ok(dy_shape, w_shape, st, pad):
    """Whether conv_dgrad takes ``pre=`` (the BN-backward apply fused into its operand loads) for this
    conv: the halo 3x3 kernel and the K = 64 panel kernel."""
    N, Ho, Wo, K = dy_shape
    Kw, R, S, C = w_shape
    return (_conv3x3_ok(N, Ho, Wo, K, C, R, S, st, pad)
            or (_s2_ok(N, 2 * Ho, 2 * Wo, C, K, R, S, st, pad, 1) and (_tuning.get("s2_halo") & 16) != 0)
            or (_panel_dgrad_k(K) and _panel_ok(N * Ho * Wo, K, C, R, S, st, pad)))


def dgrad_weight(dy_shape, w, x_shape, st, pad):
    """The transformed weight conv_dgrad builds on entry for this data gradient (tap-flipped transposed 3x3
    weight for the halo kernel, transposed 1x1 weight for the panel / A-stationary kernel), or None when its
    route takes the weight as is.  Pass it back as ``conv_dgrad(..., wprep=...)``: the fused blocks make it
    in the forward on the side stream, off the backward's critical path."""
    N, Ho, Wo, K = dy_shape
    _, H, W, C = x_shape
    Kw, R, S, C2 = w.shape
    if _conv3x3_ok(N, Ho, Wo, K, C, R, S, st, pad) or _s2_ok(N, H, W, C, K, R, S, st, pad, 1):
        return conv3x3_flip(w)
    if _panel_dgrad_k(K) and _panel_ok(N * H * W, K, C, R, S, st, pad):
        return transpose_bf16(w.view(K, C))
    return None


def conv_dgrad(dy, w, x_shape, st, pad, res=None, bn=None, out=None, res_mask=None, pre=None, wprep=None):
    """dx = conv_transpose(dy, w) (+ res).  ``out`` may alias ``res`` (in-place accumulation: for a strided
    conv only the pixels its taps reach are touched, the others keep ``res``).

    bn = (t, mean, invstd, mscale, mshift): fuse the BatchNorm backward of the layer that produced t:
    returns (gm, slab) where gm = dx * [t*mscale + mshift > 0] and slab holds the partial sums of gm and
    gm*(t-mean)*invstd (finalize with bn_bwd_finalize).

    res_mask: uint8 [N*H*W][C/8] ReLU bits (bn_apply's mask): the residual is added only where its bit is set,
    i.e. res * mask -- the identity branch's gradient computed here instead of materialised by the BN
    backward (stride 1 only).

    pre = (t, mean, invstd, gamma, dgamma, dbeta, dt_out): ``dy`` is the masked gradient gm of a BatchNorm
    whose backward apply (bn_bwd_apply mode 0) runs inside this conv's operand loads; dt_out (optional)
    receives that dt for the weight gradient.  Only where dgrad_pre_ok().

    wprep: dgrad_weight()'s result for this call (else it is made here)."""
    _bf16_c(dy, "conv_dgrad.dy")
    N, H, W, C = x_shape
    _bf16_c(w, "conv_dgrad.w")
    K, R, S, C2 = w.shape
    _chk(C2 == C, "conv_dgrad: weight [K][R][S][C]")
    _, Ho, Wo, K2 = dy.shape
    _chk(K2 == K and C % 8 == 0 and K % 8 == 0, "conv_dgrad: channel mismatch")
    if out is not None:
        _chk(tuple(out.shape) == (N, H, W, C) and out.dtype == BF16 and out.is_contiguous(), "conv_dgrad: out")
        _chk(bn is None, "conv_dgrad: out with a fused BN backward")
    if bn is not None:
        _bf16_c(bn[0], "conv_dgrad.bn_x")
        _chk(tuple(bn[0].shape) == (N, H, W, C), "conv_dgrad: bn_x shape")
    if res is not None:
        _bf16_c(res, "conv_dgrad.res")
        _chk(tuple(res.shape) == (N, H, W, C), "conv_dgrad: res shape")
    if res_mask is not None:
        _chk(res is not None and st == 1 and res_mask.dtype == torch.uint8 and res_mask.is_contiguous()
             and res_mask.numel() * 8 == N * H * W * C and (out is None or out.data_ptr() != res.data_ptr()),
             "conv_dgrad: res_mask needs res, stride 1, uint8 [N*H*W][C/8], out not aliasing res")
    if _conv3x3_ok(N, Ho, Wo, K, C, R, S, st, pad):
        # dx = conv3x3(dy, W') with the tap-flipped transposed weight (stride 1: dy and dx share H x W)
        y, slab = conv3x3(dy, wprep if wprep is not None else conv3x3_flip(w), res=res, bn=bn, out=out,
                          res_mask=res_mask, pre=pre)
        return (y, slab) if bn is not None else y
    if _s2_ok(N, H, W, C, K, R, S, st, pad, 1) and res is None and out is None and (H, W) == (2 * Ho, 2 * Wo):
        # stride 2: one launch, every output parity class a 1 / 2 / 2 / 4-tap unit-offset conv of dy (conv_s2.hip)
        y, slab = conv3x3s2(dy, wprep if wprep is not None else conv3x3_flip(w), dgrad=True, bn=bn, pre=pre)
        return (y, slab) if bn is not None else y
    if _panel_dgrad_k(K) and _panel_ok(N * H * W, K, C, R, S, st, pad) and (out is None or res is not None):
        # dx[P][C] = dy[P][K] . W[K][C]: the panel kernel with the transposed weight W^T [C][K]
        y, slab = conv1x1_panel(dy.view(-1, K), wprep if wprep is not None else transpose_bf16(w.view(K, C)),
                                res=None if res is None else res.view(-1, C), res_mask=res_mask,
                                bn=None if bn is None else (bn[0].view(-1, C),) + tuple(bn[1:]),
                                out=None if out is None else out.view(-1, C), pre=pre)
        y = y.view(N, H, W, C)
        return (y, slab) if bn is not None else y
    _chk(pre is None, "conv_dgrad: pre= needs the halo 3x3 or K = 64 panel kernel (dgrad_pre_ok)")
    dx = out if out is not None else torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    slab = None
    t = mean = inv = msc = msh = None
    if bn is not None:
        t, mean, inv, msc, msh = bn
        slab = stat_bins(C, dy.device)
    if res is not None:
        _bf16_c(res, "conv_dgrad.res")
        _chk(tuple(res.shape) == (N, H, W, C), "conv_dgrad: res shape")
    call("pdnn_conv_dgrad", ptr(dy), ptr(w), ptr(dx), N, H, W, C, K, R, S, st, pad, Ho, Wo, ptr(slab), ptr(res),
         ptr(res_mask), ptr(t), ptr(mean), ptr(inv), ptr(msc), ptr(msh), stream())
    return (dx, slab) if bn is not None else dx


# 1x1 / stride-1 weight gradients with at most this many pixels run on the ping-pong engine (ResNet-50 stages
# 2-4 at bs 256; stage 1 loses there: tools/bench_wgrad1x1.py, gpurun_out/r3_38-40, stage 3/4 67/64 -> 57/48 us)
_WGRAD1X1_PP_PIX = WGRAD1X1_PP_PIX = 200704


def conv_wgrad(x, dy, R, S, st, pad, pro=None, out=None):
    """fp32 dW [K][R][S][C] (accumulated into `out` if given, else fresh zeros)."""
    _bf16_c(x, "conv_wgrad.x")
    _bf16_c(dy, "conv_wgrad.dy")
    N, H, W, C = x.shape
    _, Ho, Wo, K = dy.shape
    if out is None:
        out = torch.zeros(K, R, S, C, device=x.device, dtype=F32)
    _chk(out.shape == (K, R, S, C) and out.is_contiguous() and out.dtype == F32, "conv_wgrad: out [K][R][S][C] fp32")
    sc, sh = pro if pro is not None else (None, None)
    P = N * H * W
    if R == 3 and S == 3 and st == 1 and pad == 1 and lib().pdnn_conv3x3_wgrad_supported(N, H, W, C, K) == 1:
        # direct kernel: LDS halo + transpose reads, partials per block, then one reduce (conv3x3_wgrad.hip); the
        # prologue relu(x * sc + sh) applied as the halo is staged
        ws = torch.empty(lib().pdnn_conv3x3_wgrad_ws(N, H, W, C, K), device=x.device, dtype=F32)
        call("pdnn_conv3x3_wgrad", ptr(x), ptr(dy), ptr(out), N, H, W, C, K, ptr(ws), ptr(sc), ptr(sh), stream())
        return out
    if (R == 3 and S == 3 and st == 2 and pad == 1 and (_tuning.get("s2_halo") & 8) != 0
            and lib().pdnn_conv3x3s2_wgrad_supported(N, H, W, C, K) == 1):
        # stride 2: the direct kernel over the input's four parity planes (conv3x3_wgrad.hip conv3x3s2_wgrad_kernel)
        ws = torch.empty(lib().pdnn_conv3x3s2_wgrad_ws(N, H, W, C, K), device=x.device, dtype=F32)
        call("pdnn_conv3x3s2_wgrad", ptr(x), ptr(dy), ptr(out), N, H, W, C, K, ptr(ws), ptr(sc), ptr(sh), stream())
        return out
    if (pro is None and R == 1 and S == 1 and st == 1 and pad == 0 and P <= _tuning.get("wgrad1x1_pp_pix")
            and P % 32 == 0 and K % 8 == 0 and C % 8 == 0):
        # plain GEMM dW[K][C] = dy[P][K]^T . x[P][C] on the ping-pong engine (split-K slabs, split count from
        # the long-reduction model): ResNet stages 2-4 (tools/bench_wgrad1x1.py, gpurun_out/r3_33, r3_38).  The joint
        # width/split plan (pdnn_pp_wgrad_plan) is faster per call in isolation (stage-2 conv1 83 -> 68 us,
        # dev/probes/wgrad1x1_sweep.py) but 1% slower end to end beside the data-gradient chain (r5_36-37)
        pp_wgrad(dy.view(P, K), x.view(P, C), out.view(K, C), splits=lib().pdnn_pp_wgrad_splits_long(K, C, P))
        return out
    call("pdnn_conv_wgrad", ptr(x), ptr(dy), ptr(out), N, H, W, C, K, R, S, st, pad, Ho, Wo, ptr(sc), ptr(sh),
         stream())
    return out


# ----------------------------------------------------------------------------------- BatchNorm
# BatchNorm statistics slabs are STAT_BINS bin-row pairs [64][2][C] fp32 that the producing kernels ADD into
# (common.h stat_add) and the finalize kernels read and zero again.  A slab therefore has to start zeroed: they
# come from a free list per (device, stream, C), refilled by bn_finalize / bn_bwd_finalize after they launch the
# zeroing finalize on that stream (a later producer on the same stream runs after it).  A slab read some other
# way (tests) is simply not returned; new ones are allocated zeroed.
STAT_BINS = 64
_BINS = {}


def _bins_key(device, C):
    # the raw stream handle (no torch.cuda.Stream object: ~100 of these per step sit on the host's critical path
    # in the forward, which the GPU can outrun)
    return (device.index, stream() if device.index == _CUR_DEV() else torch.cuda.current_stream(device).cuda_stream, C)


def stat_bins(C, device):
    """A zeroed [2 * STAT_BINS][C] fp32 statistics slab for a producer launched on the current stream."""
    free = _BINS.get(_bins_key(device, C))
    slab = free.pop() if free else torch.zeros(2 * STAT_BINS, C, device=device, dtype=F32)
    slab._pdnn_bins = "taken"
    return slab


def _release_bins(slab):
    # only slabs handed out by stat_bins, and each once (a slab finalized twice must not enter the list twice)
    if getattr(slab, "_pdnn_bins", None) != "taken":
        return
    slab._pdnn_bins = "free"
    _BINS.setdefault(_bins_key(slab.device, slab.shape[1]), []).append(slab)


def bn_finalize(slab, rows, L, eps, momentum, gamma, beta, run_mean, run_var):
    C = slab.shape[1]
    mean = torch.empty(C, device=slab.device, dtype=F32)
    invstd = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    shift = torch.empty_like(mean)
    _chk(rows == STAT_BINS and slab.shape[0] == 2 * STAT_BINS, "bn_finalize: a stat_bins() slab")
    call("pdnn_bn_finalize", ptr(slab), rows, C, float(L), float(eps), float(momentum), ptr(gamma), ptr(beta),
         ptr(run_mean), ptr(run_var), ptr(mean), ptr(invstd), ptr(scale), ptr(shift), stream())
    _release_bins(slab)
    return mean, invstd, scale, shift


def bn_eval_coeff(eps, gamma, beta, rm, rv):
    C = rm.numel()
    scale = torch.empty(C, device=rm.device, dtype=F32)
    shift = torch.empty_like(scale)
    call("pdnn_bn_eval_coeff", C, float(eps), ptr(gamma), ptr(beta), ptr(rm), ptr(rv), ptr(scale), ptr(shift),
         stream())
    return scale, shift


def bn_stats(x2d):
    L, C = x2d.shape
    _chk(C % 8 == 0 and C <= 2048, f"bn_stats: C={C}")
    slab = stat_bins(C, x2d.device)
    call("pdnn_bn_stats", ptr(x2d), L, C, ptr(slab), stream())
    return slab, STAT_BINS


def bn_apply(x2d, scale, shift, res=None, rscale=None, rshift=None, relu=True, out=None, want_mask=None):
    """y = act(x*scale + shift (+ res | res*rscale + rshift)).  With ``want_mask`` given the result is a
    pair (y, bits): bits = the sign bits of y, uint8 [L][C/8], when want_mask is true (ReLU only; the
    backward's mask mode 3 reads them instead of y), else None."""
    L, C = x2d.shape
    if out is None:
        out = torch.empty_like(x2d)
    mbits = None
    if want_mask:
        _chk(relu and C % 8 == 0, "bn_apply: mask bits need ReLU and C % 8 == 0")
        mbits = torch.empty(L, C // 8, device=x2d.device, dtype=torch.uint8)
    call("pdnn_bn_apply", ptr(x2d), L, C, ptr(scale), ptr(shift), ptr(res), ptr(rscale), ptr(rshift), int(relu),
         ptr(out), ptr(mbits), stream())
    return out if want_mask is None else (out, mbits)


def bn_bwd_reduce(g, x, mean, invstd, mode=0, msrc=None, mscale=None, mshift=None, x2=None, mean2=None,
                  invstd2=None):
    L, C = x.shape
    slab = stat_bins(C, x.device)
    slab2 = stat_bins(C, x.device) if x2 is not None else None
    call("pdnn_bn_bwd_reduce", ptr(g), ptr(x), L, C, ptr(mean), ptr(invstd), int(mode), ptr(msrc), ptr(mscale),
         ptr(mshift), ptr(slab), ptr(x2), ptr(mean2), ptr(invstd2), ptr(slab2), stream())
    return slab, slab2, STAT_BINS


def bn_bwd_finalize(slab, rows, dgamma=None, dbeta=None, accumulate=False, acc=None):
    """-> (dgamma, dbeta) of this backward; ``acc`` = (gamma.grad, beta.grad) also receive them (+=)."""
    C = slab.shape[1]
    if dgamma is None:
        dgamma = torch.empty(C, device=slab.device, dtype=F32)
        dbeta = torch.empty_like(dgamma)
    ga, ba = acc if acc is not None else (None, None)
    _chk(rows == STAT_BINS and slab.shape[0] == 2 * STAT_BINS, "bn_bwd_finalize: a stat_bins() slab")
    call("pdnn_bn_bwd_finalize", ptr(slab), rows, C, ptr(dgamma), ptr(dbeta), int(accumulate), ptr(ga), ptr(ba),
         stream())
    _release_bins(slab)
    return dgamma, dbeta


def bn_bwd_apply(g, x, mean, invstd, gamma, dgamma, dbeta, mode=0, msrc=None, mscale=None, mshift=None,
                 want_dx=True, x2=None, mean2=None, invstd2=None, gamma2=None, dgamma2=None, dbeta2=None,
                 want_gm=False):
    dx = torch.empty_like(x) if want_dx else None
    dx2 = torch.empty_like(x) if x2 is not None else None
    gm = torch.empty_like(x) if want_gm else None
    L, C = x.shape
    call("pdnn_bn_bwd_apply", ptr(g), ptr(x), L, C, ptr(mean), ptr(invstd), ptr(gamma), ptr(dgamma), ptr(dbeta),
         int(mode), ptr(msrc), ptr(mscale), ptr(mshift), ptr(dx), ptr(x2), ptr(mean2), ptr(invstd2), ptr(gamma2),
         ptr(dgamma2), ptr(dbeta2), ptr(dx2), ptr(gm), stream())
    return dx, dx2, gm


# ----------------------------------------------------------------------------------- pooling
# ImageNet stem router (tests compare the paths): 2 = the direct kernel reading the NCHW batch (default), 1 = the
# direct kernel on a channel-padded NHWC copy, 0 = the implicit-GEMM conv + bn_apply + max-pool
_STEM = {"mode": 2}


def set_stem_mode(mode: int) -> int:
    old = _STEM["mode"]
    _STEM["mode"] = int(mode)
    return old


def stem_ok(x_shape, w_shape, st, pad):
    """The ImageNet stem conv (7x7 / stride 2 / pad 3, 8 padded input channels, 64 outputs) on the direct
    stem kernel (csrc/kernels/stem.hip)."""
    return tuple(w_shape) == (64, 7, 7, 8) and x_shape[-1] == 8 and st == 2 and pad == 3 and _STEM["mode"] >= 1


def stem_conv(x, w, want_stats=True):
    """t = conv7x7/s2/p3(x) (x NHWC bf16 with 8 channels, w bf16 [64][7][7][8]) + BN partial statistics."""
    _bf16_c(x, "stem.x")
    _bf16_c(w, "stem.w")
    N, H, W, C = x.shape
    _chk(C == 8 and tuple(w.shape) == (64, 7, 7, 8), "stem_conv: x [N][H][W][8], w [64][7][7][8]")
    Ho, Wo = conv_out_hw(H, W, 7, 7, 2, 3)
    y = torch.empty(N, Ho, Wo, 64, device=x.device, dtype=BF16)
    slab = None
    if want_stats:
        slab = stat_bins(64, x.device)
    call("pdnn_stem_conv", ptr(x), ptr(w), ptr(y), N, H, W, Ho, Wo, ptr(slab), stream())
    return y, slab


def stem_nchw_ok(x):
    """The stem conv reading the NCHW bf16 batch directly (3 channels, even width >= 8)."""
    return (x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and x.shape[3] % 2 == 0 and x.shape[3] >= 8
            and _STEM["mode"] == 2)


def stem_conv_nchw(x, w32, want_stats=True):
    """t = conv7x7/s2/p3(x) for x NCHW bf16 [N][3][H][W]; w32 = stem_weight_nchw(w) bf16 [64][7][32]."""
    _bf16_c(x, "stem.x")
    _bf16_c(w32, "stem.w32")
    N, C, H, W = x.shape
    _chk(C == 3 and tuple(w32.shape) == (64, 7, 32), "stem_conv_nchw: x [N][3][H][W], w [64][7][32]")
    Ho, Wo = conv_out_hw(H, W, 7, 7, 2, 3)
    y = torch.empty(N, Ho, Wo, 64, device=x.device, dtype=BF16)
    slab = None
    if want_stats:
        slab = stat_bins(64, x.device)
    call("pdnn_stem_conv_nchw", ptr(x), ptr(w32), ptr(y), N, H, W, Ho, Wo, ptr(slab), stream())
    return y, slab


def stem_wgrad_nchw(x, dt, pre=None, acc=None):
    """Weight gradient of stem_conv_nchw: x NCHW bf16 [N][3][H][W], dt bf16 [N][Ho][Wo][64] -> fp32 [64][3][7][7]
    (a view of the kernel's [64][7 r][32 k] result, k = c*8 + j, tap s = j - 1).  pre = (t, mean, invstd, gamma,
    dgamma, dbeta, mscale, mshift): ``dt`` is the gradient of the BN+ReLU output and the BN backward apply (ReLU
    mask recomputed from t) runs inside the kernel's staging.  acc: fp32 [64, 3, 7, 7] channels-last gradient the
    result is added into (returns None)."""
    _bf16_c(x, "stem_wgrad.x")
    _bf16_c(dt, "stem_wgrad.dt")
    N, C, H, W = x.shape
    Ho, Wo = conv_out_hw(H, W, 7, 7, 2, 3)
    _chk(C == 3 and tuple(dt.shape) == (N, Ho, Wo, 64), "stem_wgrad_nchw: x [N][3][H][W], dt [N][Ho][Wo][64]")
    ws = torch.empty(lib().pdnn_stem_wgrad_ws(N, Ho, Wo), device=x.device, dtype=F32)
    if acc is not None:
        _chk(acc.dtype == F32 and tuple(acc.shape) == (64, 3, 7, 7) and acc.stride() == (147, 1, 21, 3),
             "stem_wgrad_nchw: acc fp32 [64,3,7,7] channels-last")
    dw32 = torch.empty(64, 7, 32, device=x.device, dtype=F32) if acc is None else None
    pa = (None,) * 8 if pre is None else pre
    if pre is not None:
        _bf16_c(pre[0], "stem_wgrad.t")
        _chk(tuple(pre[0].shape) == tuple(dt.shape), "stem_wgrad_nchw: t like dt")
    call("pdnn_stem_wgrad_nchw", ptr(x), ptr(dt), ptr(dw32), N, H, W, Ho, Wo, ptr(ws), *map(ptr, pa), ptr(acc),
         stream())
    if acc is not None:
        return None
    return dw32.view(64, 7, 4, 8)[:, :, :3, 1:].permute(0, 2, 1, 3)


def stem_weight_nchw(w):
    """[64][3][7][7] stem weight -> bf16 [64][7 r][32]: k = c*8 + j holds w[n][c][r][j-1] (j = 1..7, c < 3),
    zero elsewhere (the reduction order of stem_conv_nchw)."""
    k = torch.zeros(w.shape[0], 7, 4, 8, device=w.device, dtype=BF16)
    k[:, :, :3, 1:] = w.detach().permute(0, 2, 1, 3).to(BF16)
    return k.view(w.shape[0], 7, 32)


def bn_relu_maxpool(t, scale, shift):
    """(y, idx) = maxpool3x3/s2/p1(relu(t * scale + shift)) without materialising the activation; bitwise
    equal to bn_apply(relu=True) followed by maxpool_fwd."""
    _bf16_c(t, "bn_relu_maxpool.t")
    N, H, W, C = t.shape
    _chk(C % 8 == 0, "bn_relu_maxpool: C % 8")
    Ho, Wo = conv_out_hw(H, W, 3, 3, 2, 1)
    y = torch.empty(N, Ho, Wo, C, device=t.device, dtype=BF16)
    idx = torch.empty(N, Ho, Wo, C, device=t.device, dtype=torch.uint8)
    call("pdnn_bn_relu_maxpool", ptr(t), ptr(scale), ptr(shift), ptr(y), ptr(idx), N, H, W, C, Ho, Wo, stream())
    return y, idx


def maxpool_fwd(x, k, st, pad):
    _bf16_c(x, "maxpool.x")
    N, H, W, C = x.shape
    _chk(C % 8 == 0, "maxpool: C % 8")
    Ho, Wo = conv_out_hw(H, W, k, k, st, pad)
    y = torch.empty(N, Ho, Wo, C, device=x.device, dtype=BF16)
    idx = torch.empty(N, Ho, Wo, C, device=x.device, dtype=torch.uint8)
    call("pdnn_maxpool_fwd", ptr(x), ptr(y), ptr(idx), N, H, W, C, Ho, Wo, k, st, pad, stream())
    return y, idx


def maxpool_bwd(dy, idx, x_shape, k, st, pad):
    N, H, W, C = x_shape
    _, Ho, Wo, _ = dy.shape
    dx = torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    call("pdnn_maxpool_bwd", ptr(dy.contiguous()), ptr(idx), ptr(dx), N, H, W, C, Ho, Wo, k, st, pad, stream())
    return dx


def stream_wait(waiter, signaler):
    """``waiter.wait_stream(signaler)`` (same device) through a fence-free HIP event (streams.hip): no
    system-scope cache write-back at each of the ~70 fork / join points of a step (torch's wait_stream:
    10,604-10,615 vs 10,687-10,689 img/s, gpurun_out/r3_58)."""
    if waiter.device == signaler.device:
        if waiter.device.index == torch.cuda.current_device():
            call("pdnn_stream_wait", waiter.cuda_stream, signaler.cuda_stream)
        else:
            with torch.cuda.device(waiter.device):
                call("pdnn_stream_wait", waiter.cuda_stream, signaler.cuda_stream)
    else:
        waiter.wait_stream(signaler)


def maxpool_bwd_bnred(dy, idx, t, mean, invstd, mscale, mshift):
    """Stem backward: 3x3/s2/p1 max-pool gather fused with the mode-2 BN-backward reduce (mask = t*mscale +
    mshift > 0).  -> (ga [N,2Ho,2Wo,C], slab, rows) like maxpool_bwd + bn_bwd_reduce(mode=2); None when the
    shape is not covered (odd H/W, C not dividing the block)."""
    N, H, W, C = t.shape
    _, Ho, Wo, _ = dy.shape
    if H != 2 * Ho or W != 2 * Wo:
        return None
    rows = lib().pdnn_maxpool_bwd_bnred_rows(N, Ho, Wo, C)
    if rows <= 0:
        return None
    ga = torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    slab = stat_bins(C, dy.device)
    call("pdnn_maxpool_bwd_bnred", ptr(dy.contiguous()), ptr(idx), ptr(ga), ptr(t), ptr(mean), ptr(invstd),
         ptr(mscale), ptr(mshift), ptr(slab), N, Ho, Wo, C, stream())
    return ga, slab, STAT_BINS


def avgpool_fwd(x):
    _bf16_c(x, "avgpool.x")
    N, H, W, C = x.shape
    _chk(C % 8 == 0 and C <= 2048, "avgpool: C")
    y = torch.empty(N, C, device=x.device, dtype=BF16)
    call("pdnn_avgpool_fwd", ptr(x), ptr(y), N, H * W, C, stream())
    return y


def avgpool_bwd(dy, x_shape):
    N, H, W, C = x_shape
    dx = torch.empty(N, H, W, C, device=dy.device, dtype=BF16)
    call("pdnn_avgpool_bwd", ptr(dy.contiguous()), ptr(dx), N, H * W, C, stream())
    return dx


# ----------------------------------------------------------------------------------- loss
def xent_fwd(logits, labels, ignore_index=-100):
    R, V = logits.shape
    _chk(logits.stride(1) == 1, "xent: row-major logits")
    dt = 1 if logits.dtype == BF16 else 0
    _chk(logits.dtype in (BF16, F32), "xent: bf16/fp32 logits")
    loss = torch.empty(R, device=logits.device, dtype=F32)
    lse = torch.empty(R, device=logits.device, dtype=F32)
    acc = torch.empty(2, device=logits.device, dtype=F32)          # [loss sum, valid-label count], set by the call
    call("pdnn_xent_fwd", ptr(logits), logits.stride(0), R, V, ptr(labels), int(ignore_index), ptr(loss), ptr(lse),
         ptr(acc), ptr(acc[1:]), dt, stream())
    return loss, lse, acc


def xent_fwd_grad_ok(logits):
    """Whether xent_fwd_grad takes these logits (bf16, row-major, 16-byte rows, V <= 51200)."""
    R, V = logits.shape
    return (logits.dtype == BF16 and logits.stride(1) == 1 and V % 8 == 0 and logits.stride(0) % 8 == 0
            and V <= 51200 and logits.data_ptr() % 16 == 0)


def xent_fwd_grad(logits, labels, ignore_index=-100, out=None):
    """Training forward of the cross-entropy that also writes d logits = softmax - onehot, UNSCALED (the caller
    applies grad_out / count downstream), into ``out`` (default: in place over ``logits``).  One read and one
    write of the logits instead of the forward's read plus the backward's read and write.  Returns
    (loss per row, lse, acc = [loss sum, valid-label count], dlogits)."""
    _chk(xent_fwd_grad_ok(logits), "xent_fwd_grad: bf16 row-major logits, V % 8 == 0, V <= 51200")
    R, V = logits.shape
    d = logits if out is None else out
    _chk(d.shape == logits.shape and d.dtype == BF16 and d.stride(1) == 1 and d.stride(0) % 8 == 0
         and d.data_ptr() % 16 == 0, "xent_fwd_grad: bf16 row-major output")
    loss = torch.empty(R, device=logits.device, dtype=F32)
    lse = torch.empty(R, device=logits.device, dtype=F32)
    acc = torch.empty(2, device=logits.device, dtype=F32)
    call("pdnn_xent_fwd_grad", ptr(logits), logits.stride(0), R, V, ptr(labels), int(ignore_index), ptr(loss),
         ptr(lse), ptr(acc), ptr(acc[1:]), ptr(d), d.stride(0), stream())
    return loss, lse, acc, d


def xent_bwd(logits, labels, lse, gscale_dev, denom, ignore_index=-100, count=None):
    """d logits = softmax - onehot, times gscale_dev[0] / denom, or gscale_dev[0] / max(count[0], 1) with
    ``count`` (fp32 device scalar: xent_fwd's count of non-ignored rows, the mean reduction)."""
    R, V = logits.shape
    d = torch.empty_like(logits)
    dt = 1 if logits.dtype == BF16 else 0
    _chk(gscale_dev.dtype == F32 and gscale_dev.is_cuda, "xent_bwd: fp32 device gscale")
    call("pdnn_xent_bwd", ptr(logits), logits.stride(0), R, V, ptr(labels), int(ignore_index), ptr(lse),
         ptr(gscale_dev), float(denom), ptr(count), ptr(d), d.stride(0), dt, stream())
    return d


# ----------------------------------------------------------------------------------- elementwise
ACT = {"relu": 0, "sigmoid": 1, "gelu": 2, "identity": 3}


def act_fwd(x, op):
    _bf16_c(x, "act.x")
    _chk(x.numel() % 8 == 0, "act: numel % 8")
    y = torch.empty_like(x)
    call("pdnn_act_fwd", ptr(x), ptr(y), x.numel(), ACT[op], stream())
    return y


def act_bwd(g, x, op):
    g = g.contiguous()
    dx = torch.empty_like(x)
    call("pdnn_act_bwd", ptr(g), ptr(x), ptr(dx), x.numel(), ACT[op], stream())
    return dx


def add(a, b, alpha=1.0, beta=1.0, out=None):
    out = torch.empty_like(a) if out is None else out
    call("pdnn_add", ptr(a), ptr(b.contiguous()), ptr(out), a.numel(), float(alpha), float(beta), stream())
    return out


def nchw_to_nhwc(x, cpad):
    N, C, H, W = x.shape
    x = x.contiguous()
    y = torch.empty(N, H, W, cpad, device=x.device, dtype=BF16)
    call("pdnn_nchw_to_nhwc", ptr(x), int(x.dtype == BF16), ptr(y), N, C, H * W, cpad, stream())
    return y


def nhwc_to_nchw_f32(x, C):
    N, H, W, Cp = x.shape
    y = torch.empty(N, C, H, W, device=x.device, dtype=F32)
    call("pdnn_nhwc_to_nchw_f32", ptr(x), ptr(y), N, C, H * W, Cp, stream())
    return y


def colsum(x2d, out=None, accumulate=False, deterministic=False):
    """out[C] (fp32) = (or +=) column sums of a bf16 [R][C] matrix.  Accumulating into ``out`` takes the
    one-launch atomic form (no partial rows / level-2 kernel; add order varies) unless ``deterministic``."""
    R, C = x2d.shape
    x2d = x2d.contiguous()
    if out is None:
        out = torch.empty(C, device=x2d.device, dtype=F32)
    work = None
    if C % 8 == 0 and R > 256 and (deterministic or not accumulate):
        work = torch.empty(lib().pdnn_colsum_splits(R) * C, device=x2d.device, dtype=F32)
    call("pdnn_colsum", ptr(x2d), R, C, ptr(out), int(accumulate), ptr(work), stream())
    return out


# ----------------------------------------------------------------------------------- optim / buckets
def sgd_step(p, g, buf, shadow, lr, momentum, dampening, wd, nesterov, gscale_dev=None, gscale=1.0, first=False,
             hyper=None):
    """``hyper`` (optional fp32 device tensor [lr]) overrides ``lr`` at run time (graph replay)."""
    call("pdnn_sgd_step", ptr(p), ptr(g), ptr(buf), ptr(shadow), p.numel(), float(lr), float(momentum),
         float(dampening), float(wd), int(nesterov), ptr(gscale_dev), float(gscale), int(first), ptr(hyper), stream())


def adam_step(p, g, m, v, shadow, lr, b1, b2, eps, wd, decoupled, bc1, bc2, gscale_dev=None, gscale=1.0, hyper=None):
    """``hyper`` (optional fp32 device tensor [lr, 1-b1^t, 1-b2^t]) overrides lr/bc1/bc2 (graph replay)."""
    call("pdnn_adam_step", ptr(p), ptr(g), ptr(m), ptr(v), ptr(shadow), p.numel(), float(lr), float(b1), float(b2),
         float(eps), float(wd), int(decoupled), float(bc1), float(bc2), ptr(gscale_dev), float(gscale), ptr(hyper),
         stream())


def cast_f32_bf16(x, y, scale=1.0):
    call("pdnn_cast_f32_bf16", ptr(x), ptr(y), x.numel(), float(scale), stream())


def cast_bf16_f32(x, y, scale=1.0, accumulate=False):
    call("pdnn_cast_bf16_f32", ptr(x), ptr(y), x.numel(), float(scale), int(accumulate), stream())


def scale_(x, scale=1.0, dev_scale=None, invert=False):
    call("pdnn_scale_f32", ptr(x), x.numel(), float(scale), ptr(dev_scale), int(invert), stream())


def axpy_(y, x, a):
    call("pdnn_axpy_f32", ptr(y), ptr(x), y.numel(), float(a), stream())


def sumsq(x, out):
    call("pdnn_sumsq_f32", ptr(x), x.numel(), ptr(out), stream())
    return out


# ----------------------------------------------------------------------------------- transformer
def gemm_batched(a, lda, sa, amode, b, ldb, sb, bmode, c, ldc, sc, M, N, K, nb, alpha=1.0, res=None, causal=0):
    """Strided batched GEMM over nb = (nb1, nb2) batches: C = alpha * A . B (+res).

    amode 0: A[M][K] row stride lda; 1: A stored [K][M].  bmode 0: B stored [N][K]; 1: B stored [K][N].
    sa/sb/sc = (stride1, stride2) in elements.  ``c`` is a bf16 or fp32 tensor (base pointer)."""
    _chk(lda % 8 == 0 and ldb % 8 == 0 and K % 8 == 0, "gemm_batched: 16-byte aligned leading dims")
    _chk(all(s % 8 == 0 for s in (*sa, *sb)), "gemm_batched: 16-byte aligned batch strides")
    _chk(c.dtype in (BF16, F32), "gemm_batched: bf16/fp32 output")
    call("pdnn_gemm_batched", int(amode), int(bmode), int(c.dtype == F32), ptr(a), lda, sa[0], sa[1], ptr(b), ldb,
         sb[0], sb[1], ptr(c), ldc, sc[0], sc[1], M, N, K, nb[0], nb[1], float(alpha), ptr(res), int(causal),
         stream())
    return c


def gemm_nt_ex(x, w, bias=None, act=0, aux=None, res=None, dgelu=None, w_kn=False, out=None):
    """y = act(x @ w^T + bias) (+res); act 0/1/2 = none/ReLU/GELU(tanh), GELU also stores the
    pre-activation into ``aux``; ``dgelu``: y *= gelu'(dgelu).  ``w_kn``: w stored [K][N] (y = x @ w)."""
    M, K = x.shape
    N = w.shape[1] if w_kn else w.shape[0]
    _chk((w.shape[0] if w_kn else w.shape[1]) == K and K % 8 == 0 and N % 8 == 0, f"gemm_nt_ex: {x.shape} {w.shape}")
    _chk(x.stride(1) == 1 and w.is_contiguous() and x.stride(0) % 8 == 0, "gemm_nt_ex: row-major operands")
    if out is None:
        out = torch.empty(M, N, device=x.device, dtype=BF16)
    for t in (aux, res, dgelu):
        _chk(t is None or (t.shape == out.shape and t.stride() == out.stride()), "gemm_nt_ex: epilogue operand shape")
    call("pdnn_gemm_nt_ex", ptr(x), x.stride(0), ptr(w), w.stride(0), ptr(out), out.stride(0), M, N, K, 1.0,
         ptr(bias), int(act), ptr(aux), ptr(res), ptr(dgelu), int(w_kn), stream())
    return out


def layernorm_fwd(x, g, b, eps):
    _bf16_c(x, "layernorm.x")
    R, D = x.shape
    _chk(D % 8 == 0 and D <= 2048, f"layernorm: D={D}")
    y = torch.empty_like(x)
    mean = torch.empty(R, device=x.device, dtype=F32)
    rstd = torch.empty_like(mean)
    call("pdnn_layernorm_fwd", ptr(x), ptr(g), ptr(b), ptr(y), ptr(mean), ptr(rstd), R, D, float(eps), stream())
    return y, mean, rstd


def layernorm_bwd(dy, x, g, mean, rstd, dres=None, acc=None):
    """-> dx (+dres), dgamma, dbeta; with ``acc`` = (gamma.grad, beta.grad) the parameter gradients are
    accumulated there instead (returns dx, None, None)."""
    R, D = x.shape
    dy = dy.contiguous()
    _chk(dy.shape == x.shape and (dres is None or dres.shape == x.shape), "layernorm_bwd: shapes")
    nb = lib().pdnn_layernorm_bwd_blocks(R)
    slab = stat_bins(D, x.device)
    dx = torch.empty_like(x)
    call("pdnn_layernorm_bwd", ptr(dy), ptr(x), ptr(g), ptr(mean), ptr(rstd), ptr(dres), ptr(dx), ptr(slab), R, D,
         nb, stream())
    if acc is not None:
        bn_bwd_finalize(slab, STAT_BINS, dgamma=acc[0], dbeta=acc[1], accumulate=True)
        return dx, None, None
    dg, db = bn_bwd_finalize(slab, STAT_BINS)
    return dx, dg, db


def attn_softmax_fwd(S, P, lse, rows, T, scale, causal=True):
    _chk(T % 4 == 0 and S.dtype == F32 and P.dtype == BF16 and S.numel() >= rows * T and P.numel() >= rows * T,
         "attn_softmax_fwd: buffers")
    call("pdnn_attn_softmax_fwd", ptr(S), T, ptr(P), T, ptr(lse), rows, T, float(scale), int(causal), stream())


def attn_softmax_bwd(P, dP, dS, rows, T, scale, causal=False):
    """causal: dP above the diagonal is never read (the causal dP GEMM leaves it unwritten); dS there is 0."""
    _chk(T % 4 == 0 and dP.dtype == F32 and dS.dtype == BF16, "attn_softmax_bwd: buffers")
    call("pdnn_attn_softmax_bwd", ptr(P), T, ptr(dP), T, ptr(dS), T, rows, T, float(scale), int(bool(causal)),
         stream())


def flash_attn_fwd(qkv, B, T, H, scale, causal=True):
    """Fused attention, head dim 64: qkv [B*T][3*H*64] -> (out [B*T][H*64], lse2 [B][H][T])."""
    _bf16_c(qkv, "flash_attn.qkv")
    _chk(qkv.shape == (B * T, 3 * H * 64) and T % 128 == 0, f"flash_attn: qkv {tuple(qkv.shape)} B={B} T={T} H={H}")
    out = torch.empty(B * T, H * 64, device=qkv.device, dtype=BF16)
    lse2 = torch.empty(B, H, T, device=qkv.device, dtype=F32)
    call("pdnn_flash_attn_fwd", ptr(qkv), ptr(out), ptr(lse2), B, T, H, float(scale), int(causal), stream())
    return out, lse2


def flash_attn_bwd(qkv, out, dout, lse2, B, T, H, scale, causal=True):
    dout = dout.contiguous()
    _chk(dout.shape == out.shape and lse2.shape == (B, H, T), "flash_attn_bwd: shapes")
    dqkv = torch.empty_like(qkv)
    delta = torch.empty(B, H, T, device=qkv.device, dtype=F32)
    call("pdnn_flash_attn_bwd", ptr(qkv), ptr(out), ptr(dout), ptr(lse2), ptr(delta), ptr(dqkv), B, T, H, float(scale),
         int(causal), stream())
    return dqkv


def embedding_fwd(idx, wte, wpe, T):
    R = idx.numel()
    D = wte.shape[1]
    _chk(idx.dtype == torch.int64 and idx.is_contiguous() and D % 8 == 0, "embedding: int64 ids, D % 8")
    _chk(wpe is None or (wpe.shape[1] == D and wpe.shape[0] >= T), "embedding: wpe shape")
    out = torch.empty(R, D, device=wte.device, dtype=BF16)
    call("pdnn_embedding_fwd", ptr(idx), ptr(wte), ptr(wpe), ptr(out), R, T, D, stream())
    return out


def embedding_bwd(idx, g, dwte, dwpe, T, scale=1.0):
    """dwte[idx[r]] += scale * g[r], dwpe[r % T] += g[r] (fp32 atomics); either table may be None."""
    R, D = g.shape
    _chk((dwte is None or (dwte.dtype == F32 and dwte.shape[1] == D and dwte.is_contiguous()))
         and (dwpe is None or (dwpe.dtype == F32 and dwpe.shape[1] == D and dwpe.is_contiguous()))
         and idx.dtype == torch.int64 and idx.numel() == R, "embedding_bwd")
    if dwte is None or scale != 1.0:
        call("pdnn_embedding_bwd_scaled", ptr(idx), ptr(g.contiguous()), ptr(dwte), ptr(dwpe), R, T, D, float(scale),
             stream())
        return
    call("pdnn_embedding_bwd", ptr(idx), ptr(g.contiguous()), ptr(dwte), ptr(dwpe), R, T, D, stream())


# ----------------------------------------------------------------------------------- fp8 (OCP e4m3)
U8 = torch.uint8


def fp8_probe(A, Bt, layout):
    D = torch.empty(16, 16, device=A.device, dtype=F32)
    call("pdnn_fp8_probe", ptr(A), ptr(Bt), ptr(D), int(layout), stream())
    return D


def amax_(x, out):
    """out (fp32 [1], device) = max(out, max|x|)."""
    if x.dtype == BF16:
        call("pdnn_amax_bf16", ptr(x), x.numel(), ptr(out), stream())
    else:
        call("pdnn_amax_f32", ptr(x), x.numel(), ptr(out), stream())
    return out


def fp8_scale(amax, scale, inv, margin=0):
    """scale = 448 / amax * 2^-margin (device scalars, no host sync)."""
    call("pdnn_fp8_scale", ptr(amax), ptr(scale), ptr(inv), int(margin), stream())


def fp8_scale_step(amax, scale, inv, inv_w, gemm_scale, margin=0):
    call("pdnn_fp8_scale_step", ptr(amax), ptr(scale), ptr(inv), ptr(inv_w), ptr(gemm_scale), int(margin), stream())


def fp8_scale_roll(amax, scale, inv, e5m2=False, margin=0):
    """After an in-line quantisation (conv3x3_fp8): reduce + reset the amax partials, roll the delayed scale."""
    call("pdnn_fp8_scale_roll", ptr(amax), ptr(scale), ptr(inv), int(bool(e5m2)), int(margin), stream())


def conv3x3_fp8_ok(N, H, W, C, Ko):
    """Whether the fp8 halo kernel takes this 3x3 / stride-1 / pad-1 conv (C, Ko multiples of 128)."""
    return bool(_C3["mode"]) and lib().pdnn_conv3x3_fp8_supported(N, H, W, C, Ko) == 1


def conv3x3_flip8(wq, K, C):
    """e4m3 [K][3][3][C] -> [C][3][3][K] tap-flipped (same scale): the fp8 data gradient's weight."""
    wt = torch.empty(C, 3, 3, K, device=wq.device, dtype=U8)
    call("pdnn_conv3x3_flip8", ptr(wq), ptr(wt), K, C, stream())
    return wt


def conv3x3_wgrad_fp8(x, dy, act_x, act_dy, out=None, pro=None):
    """dW [K][3][3][C] fp32 (+= into ``out``) of a 3x3 / stride-1 / pad-1 conv on the fp8 direct weight-gradient
    kernel: x quantised to e4m3 with ``act_x``'s current scale, dy to e5m2 with ``act_dy``'s (ops.fp8.Fp8Act: the
    scales the fp8 halo conv just rolled to these tensors' own |max|)."""
    _bf16_c(x, "conv3x3_wgrad_fp8.x")
    _bf16_c(dy, "conv3x3_wgrad_fp8.dy")
    N, H, W, C = x.shape
    _, Ho, Wo, K = dy.shape
    _chk((Ho, Wo) == (H, W) and lib().pdnn_conv3x3_wgrad_supported(N, H, W, C, K) == 1, "conv3x3_wgrad_fp8: shape")
    if out is None:
        out = torch.zeros(K, 3, 3, C, device=x.device, dtype=F32)
    _chk(out.shape == (K, 3, 3, C) and out.is_contiguous() and out.dtype == F32, "conv3x3_wgrad_fp8: out")
    ws = torch.empty(lib().pdnn_conv3x3_wgrad_ws(N, H, W, C, K), device=x.device, dtype=F32)
    psc, psh = pro if pro is not None else (None, None)
    call("pdnn_conv3x3_wgrad_fp8", ptr(x), ptr(dy), ptr(out), N, H, W, C, K, ptr(ws), ptr(act_x.scale),
         ptr(act_dy.scale), ptr(act_x.inv), ptr(act_dy.inv), ptr(psc), ptr(psh), stream())
    return out


def conv3x3_fp8(x, wq, winv, act, want_stats=False, bn=None, pre=None, pro=None):
    """y = conv3x3(x, w) on the fp8 halo kernel: x bf16 NHWC (quantised in the kernel's halo staging with the
    delayed scale of ``act`` -- an ops.fp8.Fp8Act, e4m3 or e5m2), wq e4m3 [N][3][3][C] with inverse scale ``winv``
    (device scalar).  Epilogues / ``bn`` / ``pre`` as conv3x3 (bn and pre only with e5m2: data gradients).
    The first call of an ``act`` runs the kernel once to measure the operand's amax."""
    _bf16_c(x, "conv3x3_fp8.x")
    Nimg, H, W, C = x.shape
    Ko = wq.shape[0]
    _chk(wq.dtype == U8 and wq.is_contiguous() and wq.numel() == Ko * 9 * C, "conv3x3_fp8: wq e4m3 [N][3][3][C]")
    y = torch.empty(Nimg, H, W, Ko, device=x.device, dtype=BF16)
    slab = None
    t = mean = inv = msc = msh = None
    if want_stats or bn is not None:
        slab = stat_bins(Ko, x.device)
    if bn is not None:
        t, mean, inv, msc, msh = bn
    def args(sl):
        return (ptr(x), ptr(wq), ptr(y), Nimg, H, W, C, Ko, ptr(sl), ptr(t), ptr(mean), ptr(inv), ptr(msc), ptr(msh),
                *_pre_args(pre, x), ptr(act.scale), ptr(act.inv), ptr(winv), ptr(act.amax), int(act.e5m2),
                ptr(pro[0] if pro is not None else None), ptr(pro[1] if pro is not None else None), stream())
    if not act.primed:
        # the priming run's statistics go to a throwaway slab (the bins are added into, not overwritten)
        call("pdnn_conv3x3_fp8", *args(stat_bins(Ko, x.device) if slab is not None else None))
        fp8_scale_roll(act.amax, act.scale, act.inv, act.e5m2, act.margin)
        act.primed = True
    call("pdnn_conv3x3_fp8", *args(slab))
    fp8_scale_roll(act.amax, act.scale, act.inv, act.e5m2, act.margin)
    return y, slab


_FP8_PARTS = {}


def quant_fp8_current(x, inv, margin=0, out=None):
    """e4m3 copy of bf16 ``x`` with current scaling (scale from x's own amax, two launches, no fill);
    ``inv`` (1 device float) receives 1 / scale."""
    _chk(x.dtype == BF16 and x.is_contiguous() and x.numel() % 8 == 0, "quant_fp8_current: contiguous bf16")
    parts = _FP8_PARTS.get(x.device)
    if parts is None:
        parts = _FP8_PARTS[x.device] = torch.empty(1024, device=x.device, dtype=F32)
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=U8)
    call("pdnn_quant_fp8_current", ptr(x), x.numel(), ptr(parts), ptr(out), ptr(inv), int(margin), stream())
    return out


def quant_fp8(x, scale, out=None, amax=None):
    """e4m3(x * scale) as uint8; bf16 input may also record its amax (delayed scaling)."""
    _chk(x.is_contiguous() and x.numel() % 8 == 0, "quant_fp8: contiguous, numel % 8")
    if out is None:
        out = torch.empty(x.shape, device=x.device, dtype=U8)
    if x.dtype == BF16:
        call("pdnn_quant_fp8", ptr(x), x.numel(), ptr(scale), ptr(out), ptr(amax), stream())
    else:
        _chk(x.dtype == F32 and amax is None, "quant_fp8: fp32 input without amax")
        call("pdnn_quant_fp8_f32", ptr(x), x.numel(), ptr(scale), ptr(out), stream())
    return out


def dequant_fp8(q, inv):
    out = torch.empty(q.shape, device=q.device, dtype=BF16)
    call("pdnn_dequant_fp8", ptr(q), q.numel(), ptr(inv), ptr(out), stream())
    return out


def gemm_fp8(xq, wq, scale, bias=None, act=0, aux=None, res=None, stats=None, out_f32=False, out=None):
    """y[M][N] = act(scale * xq[M][K] . wq[N][K]^T + bias) (+res); xq, wq e4m3 (uint8), K % 128 == 0."""
    M, Kd = xq.shape
    N, K2 = wq.shape
    _chk(xq.dtype == U8 and wq.dtype == U8 and K2 == Kd and Kd % 128 == 0 and N % 8 == 0,
         f"gemm_fp8: {tuple(xq.shape)} {tuple(wq.shape)}")
    _chk(xq.stride(1) == 1 and wq.stride(1) == 1 and xq.stride(0) % 16 == 0 and wq.stride(0) % 16 == 0,
         "gemm_fp8: K-contiguous rows, 16-byte aligned")
    if out is None:
        out = torch.empty(M, N, device=xq.device, dtype=F32 if out_f32 else BF16)
    call("pdnn_gemm_fp8", ptr(xq), xq.stride(0), ptr(wq), wq.stride(0), ptr(out), out.stride(0), M, N, Kd,
         ptr(scale), ptr(bias), int(act), ptr(aux), ptr(res), ptr(stats), int(out_f32), stream())
    return out
