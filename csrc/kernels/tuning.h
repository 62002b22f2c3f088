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
    X(glds, 1, "256-row glds engine: 0 off, 1 automatic (>= 192 output tiles; forward from K = 1024), 2 whenever " \
               "the operands allow (tests)")                                                                 \
    X(pp, 1, "ping-pong engine for plain GEMMs (and fp8): 0 off, 1 automatic, 2 whenever the operands allow (tests)") \
    X(pp_bn, 0, "force the ping-pong tile width (96/128/192/256/288; 0 automatic; tests)")                \
    X(conv3x3_force, 0, "halo 3x3 conv also for images narrower than 12 (tests)")                         \
    X(pp_dgrad_bn_k, 1024, "1x1 data gradients with the BN-backward epilogue on the ping-pong engine from this "   \
                           "reduction length (ResNet-50 conv3 stages 3-4; gpurun_out/r4_15-17)")

struct Tune {
#define PDNN_TUNE_FIELD(n, d, doc) int n = d;
    PDNN_TUNE_TABLE(PDNN_TUNE_FIELD)
#undef PDNN_TUNE_FIELD
};

Tune& tune();     // the process-wide table (PDNN_TUNE applied on first use)

}  // namespace pg
