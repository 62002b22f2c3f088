"""Python-side entries of the dispatch table (the kernel-side table is csrc/kernels/tuning.h).

One environment variable overrides either side for A/B runs: ``PDNN_TUNE="key=value,key=value"`` (keys of
both tables; the kernel library reports unknown ones when it loads).  Each default is the measured optimum:

=================  =======  ===========================================================================
key                default  meaning (measurement)
=================  =======  ===========================================================================
wide1x1_fwd        1        1x1 / stride-1 forward convs with K >= 512 input channels on the long-reduction streaming
                            kernel (conv1x1_wide.hip) instead of the implicit-GEMM engines
wide1x1_dgrad      1        ... and the 1x1 / stride-1 data gradients with K >= 512
bn3_pre            1        Bottleneck: BN3's backward apply (mode 3, the output ReLU bits) inside conv3's data-gradient
                            operand loads on that kernel instead of a separate apply pass
side_wgrad         1        conv weight gradients on a second HIP stream beside the data-gradient chain
                            (ResNet-50 +8.3%, profiles/resnet50_bs256_side_stream_r2.txt)
materialize_a2     1        Bottleneck: write a2 = relu(bn2(t2)) once instead of conv3's operand prologue
                            (9,240 -> 9,596 img/s, gpurun_out/r3_05)
conv3x3            1        3x3 / stride-1 convs on the LDS-halo kernel (+2.5%, gpurun_out/r3_07)
panel1x1           1        1x1 / stride-1 convs with K <= 128 on the pixel-panel kernel (+1.1%, r3_08)
bwd_pre            1        BatchNorm-backward apply (dt = k*gm + A*t + B) fused into the operand loads of
                            the consuming halo 3x3 / K=64 panel data gradient, dt written once for the wgrad
stem               2        ImageNet stem (stem.hip): 0 generic conv + bn_apply + max-pool, 1 direct 7x7/s2 kernel on
                            the NHWC copy + fused BN-apply/ReLU/max-pool, 2 the same reading the NCHW batch
direct_grad        1        fused ops accumulate weight gradients straight into the flat arena
bn_fused_fin       1        BatchNorm slab finalize in one launch (level-1 blocks hand their rows to the last
                            arriver through a counter, batchnorm.hip bn_slab_fused_kernel) instead of two
stem_wgrad_nchw    1        ImageNet stem weight gradient straight from the NCHW batch (stem_wgrad.hip) instead of the
                            implicit-GEMM im2col over a channel-padded NHWC copy
light_events       1        cross-stream fork / join of the two-stream ResNet step through fence-free HIP events
                            (streams.hip) instead of torch's Stream.wait_stream (system-scope release per marker);
                            off: 10,604-10,615 vs 10,687-10,689 img/s (gpurun_out/r3_58); DDP path (bucket launches
                            fork too) 10,574-10,586 vs 10,692-10,695 (r3_60)
wprep_once         1        wprep: one side-stream fork per model forward and one compute-stream wait per backward (the
                            latest transform event covers the earlier ones) instead of one of each per block;
                            off: 10,819-10,821 vs 10,844-10,853 img/s (gpurun_out/r3_73)
pool_bnred         1        stem backward: max-pool gather and the mode-2 BN-backward reduce in one pass
                            (pool.hip maxpool_bwd_bnred_kernel) instead of maxpool_bwd + bn_bwd_reduce;
                            off: 10,644-10,656 vs 10,718-10,720 img/s (gpurun_out/r3_57)
wgrad3x3           1        3x3 / stride-1 weight gradients on the direct halo kernel (conv3x3_wgrad.hip) instead of
                            the implicit-GEMM engine
wprep              1        the data gradients' transformed weights (flipped 3x3, transposed 1x1) made in the forward
                            on the side stream instead of on the backward's critical path
wgrad1x1_pp_pix    200704   1x1 / stride-1 weight gradients with at most this many pixels on the ping-pong
                            engine (ResNet-50 stages 2-4 at bs 256; stage 1 loses there, tools/bench_wgrad1x1.py,
                            gpurun_out/r3_38-40: stage 3/4 67/64 -> 57/48 us, stage 2 81 -> 60-78 us); 0 = off
=================  =======  ===========================================================================
"""
from __future__ import annotations

import os

DEFAULTS = {"wide1x1_fwd": 1, "wide1x1_dgrad": 1, "bn3_pre": 1, "side_wgrad": 1, "materialize_a2": 1, "conv3x3": 1, "panel1x1": 1, "bwd_pre": 1, "stem": 2, "direct_grad": 1, 
            "wgrad1x1_pp_pix": 200704, "bn_fused_fin": 1, "wprep": 1, "wgrad3x3": 1, "stem_wgrad_nchw": 1,
            "pool_bnred": 1, "light_events": 1, "wprep_once": 1}

_VALUES = dict(DEFAULTS)


def _parse(s: str) -> dict:
    out = {}
    for item in filter(None, (p.strip() for p in s.split(","))):
        if "=" not in item:
            raise ValueError(f"PDNN_TUNE: {item!r} is not key=value")
        k, v = item.split("=", 1)
        out[k.strip()] = int(v)
    return out


for _k, _v in _parse(os.environ.get("PDNN_TUNE", "")).items():
    if _k in _VALUES:
        _VALUES[_k] = _v


def get(key: str) -> int:
    return _VALUES[key]


def set(key: str, value: int) -> int:        # noqa: A001 - mirrors pdnn_tune_set
    """Set a Python-side entry; returns the previous value."""
    if key not in _VALUES:
        raise KeyError(f"unknown tuning key {key!r} (kernel-side keys: ops.kernels.tune_set)")
    old = _VALUES[key]
    _VALUES[key] = int(value)
    return old
