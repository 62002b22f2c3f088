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
    X(pp_sk64, 1, "96 / 128-wide ping-pong tiles with K-major operands and K % 64 == 0 (no split-K) stream 64-deep "  \
                  "slices (128-byte rows) instead of 32-deep; 0 = 32-deep")                                    \
    X(pp_epi_slack, 2, "ping-pong plain epilogues store through buffer stores (every wave issues the same count) " \
                       "and the next item's first load waits leave them in flight, so a tile's store drain overlaps " \
                       "the next item's MFMAs instead of stalling its first slice: 1 = bf16 outputs, 2 = also the "  \
                       "fp32 ones (weight gradients, split-K slabs), 0 = drain at once.  Bit-identical; LM-head "    \
                       "forward 888 -> 873 us (r6_09, r6_12); 2 vs 1: GPT-2 624.2k / 625.5k -> 632.0k / 630.9k "    \
                       "tok/s, ResNet-50 11,911 -> 11,929 img/s same box (r6_13)")                                   \
    X(pp_epi_pair, 1, "ping-pong engine: the two staggered wave groups write their tile halves in the same barrier " \
                      "interval (one extra barrier each per item) instead of one after the other beside the other " \
                      "group's compute (two epilogue-long intervals per item at one wave per SIMD).  With "         \
                      "pp_epi_slack: LM-head forward 888 -> 759 us, GPT-2 N = 768 GEMMs -10..16%, GPT-2 step "      \
                      "591k -> 622k tok/s, ResNet-50 11,835 -> 11,899 img/s same box, bit-identical (r6_12)")       \
    X(stem_wgrad_blocks, 2048, "ImageNet stem weight gradient: grid cap (fixed runs of 96-pixel tiles per block; two " \
                               "blocks fit a CU).  At 512 the kernel took 325-330 or 498-501 us inside the ResNet-50 "  \
                               "step (a launch overlapping the side stream's last kernel leaves a CU with two runs in " \
                               "sequence), 2048: 330-360 (gpurun_out/r6_26); alone 370 vs 390 us (r6_25)")              \
    X(attn_bwd_wide, 3, "flash-attention backward kernels with two 16-row fragments per wave (half the LDS "       \
                        "fragment reads per MFMA), a bit mask: 1 dQ (32 queries per wave), 2 dK / dV (32 keys per wave). " \
                        "Alone (B8 T1024 causal) 0: 87.4 us, 1: 90.1, 3: 90.3; B32: 330 / 315 / 302 us; in the GPT-2 " \
                        "step beside the side-stream weight gradients 1: 688.5k / 687.4k vs 0: 680.6k / 681.8k tok/s, " \
                        "3: 688.6k / 683.3k (gpurun_out/r6_45); three more pairs 1 vs 3: 693.1k / 696.3k, 691.0k / "  \
                        "693.2k, 693.8k / 694.0k (r6_62) -- level in the GPT-2 step, 4-9% faster alone at B32 / T4096")  \
    X(attn_delta_in_dq, 1, "flash-attention backward: the dQ kernel forms delta = rowsum(dO . O) itself and runs " \
                           "before dK / dV (0: a separate delta launch first)")                                  \
    X(conv3x3_force, 0, "halo 3x3 conv also for images narrower than 12 (tests)")                         \
    X(pp_conv_fwd_c, 512, "1x1 / stride-1 conv forwards without an operand prologue on the ping-pong engine " \
                          "(statistics epilogue) from this many input channels (1 << 20 = never: the implicit-GEMM " \
                          "engines).  ResNet-50's conv1 / shortcut forwards with C >= 512: 11,907 / 11,956 -> "     \
                          "12,015 / 12,007 img/s same box (gpurun_out/r6_16)")                                      \
    X(pp_dgrad_bn_k, 1024, "1x1 data gradients with the BN-backward epilogue on the ping-pong engine from this "   \
                           "reduction length (ResNet-50 conv3 stages 3-4; gpurun_out/r4_15-17)")                 \
    X(comm_cus, 0, "CUs the persistent grids (ping-pong GEMMs, stem) leave free for RCCL's channel blocks while " \
                   "a multi-rank process group is live (set_comm_world > 1; 0 = fill the chip). A persistent block " \
                   "holds its CU for the whole kernel, so a bucket all-reduce issued beside it waits for the GEMM to " \
                   "drain.  Priced at a forced comm world of 8 on one GPU (gpurun_out/r6_01): 16 / 8 cost GPT-2 " \
                   "4.9% / 4.7% (587.0k / 587.8k vs 617.0k tok/s: the ping-pong grids lose their whole-round fill), " \
                   "ResNet-50 0.4%; the benefit is unmeasured without a multi-GPU box, so off")

struct Tune {
#define PDNN_TUNE_FIELD(n, d, doc) int n = d;
    PDNN_TUNE_TABLE(PDNN_TUNE_FIELD)
#undef PDNN_TUNE_FIELD
};

Tune& tune();     // the process-wide table (PDNN_TUNE applied on first use)

// CUs a persistent grid may fill: the device's CU count, minus tune().comm_cus while the process is one rank of
// a multi-rank job (pdnn_set_comm_world), rounded down to whole XCDs (8 on gfx950) so the blockIdx -> XCD
// round-robin stays balanced
int grid_cus();

}  // namespace pg
