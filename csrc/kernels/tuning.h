// Dispatch table of the GEMM / convolution engines (gemm_mfma.hip, gemm_pp.hip, gemm_glds.h, conv3x3.hip).
//
// Every shape threshold and engine switch lives in ONE table, with the default that measured best and the
// run that chose it.  There are no per-knob environment variables: an A/B run overrides entries through the
// single variable PDNN_TUNE="key=value,key=value" (read once, unknown keys reported by pdnn_tune_error())
// or pdnn_tune_set(); the GPU test tests/test_tuning_gpu.py runs the kernels under every entry's
// alternative values.
#pragma once

namespace pg {

// X(name, default, doc)
#define PDNN_TUNE_TABLE(X)                                                                                    \
    X(glds, 1, "256-row glds engine: 0 off, 1 automatic (grid size and shape below), 2 whenever the operands " \
               "allow (tests)")                                                                              \
    X(glds_min_tiles, 192, "glds only with >= this many output tiles (r1 sweep, profiles/glds_threshold_sweep)") \
    X(glds_fwd_k, 1024, "implicit-GEMM conv forward on glds from this reduction length (r1: 512/1024/never tie)") \
    X(glds_dgrad_n, 1 << 30, "conv data gradient on glds from this many input channels (off: r1 whole-step -2.3%)") \
    X(glds_dgrad_k, 1 << 30, "conv data gradient on glds from this reduction length (off, as above)")         \
    X(pp, 1, "ping-pong engine for plain GEMMs: 0 off, 1 automatic, 2 whenever the operands allow (tests)")      \
    X(pp_bn, 0, "force the ping-pong tile width (96/128/192/256/288; 0 automatic)")                        \
    X(pp_fp8, 1, "fp8 GEMMs on the ping-pong engine (0: glds engine)")                                      \
    X(pp_conv_min_n, 128, "1x1 stride-1 convs on the ping-pong engine from this output width")               \
    X(pp_conv_fwd_k, 1 << 30, "... forward from this reduction length (off: BN-stats epilogue slower there)")  \
    X(pp_conv_dgrad_k, 512, "... data gradient from this reduction length (r2_46: 512 vs 256 +0.5%)")        \
    X(pp_conv_bnb_k, 1 << 30, "... data gradient with the fused BN-backward epilogue from this reduction length")  \
    X(staged_store, 1, "128-row kernel: bf16 epilogue stores staged through LDS (full rows)")                \
    X(lowk_bn64, 24, "GEMMs of <= this many K-steps take the 128x64 tile (r2_42-44 sweep: 24)")             \
    X(split_blocks, 512, "split-K weight gradients: target blocks (r2 sweep: 256/384 -2%/-1%, 768 equal)")   \
    X(conv3x3_force, 0, "halo 3x3 conv also for images narrower than 12 (tests)")                           \
    X(areg, 2, "A-stationary 1x1 kernel: 0 off, 1 for K = 256 (LDS panel for K <= 128), 2 for every K <= 256 " \
               "(r3_15: 9,844 vs 9,780 / 9,690 img/s for 1 / 0)")

struct Tune {
#define PDNN_TUNE_FIELD(n, d, doc) int n = d;
    PDNN_TUNE_TABLE(PDNN_TUNE_FIELD)
#undef PDNN_TUNE_FIELD
};

Tune& tune();     // the process-wide table (PDNN_TUNE applied on first use)

}  // namespace pg
