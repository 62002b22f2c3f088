// 1x1 / stride-1 convolutions with a LONG reduction (K = C_in in {512, 1024, 2048}) on MFMA (gfx950):
// y[P][N] = x[P][K] . W[N][K]^T.  In ResNet-50 these are the data gradients of conv3 (dt3 [P][4w] -> [P][w],
// with the BatchNorm-backward epilogue of BN2) in stages 2-4 and of conv1 in stage 4, and the stage-3/4
// forward convs with K >= 512.  On the 128-row implicit-GEMM engine they ran at 9.5-14% of the bf16 peak,
// 2-3x their HBM floor (profiles/resnet50_bs256_pmc_r3_end.txt: 2.95 ms/step).
//
// They are memory-bound (every activation byte feeds 2 * NB flops, NB <= 512 output columns; the HBM
// floor is the x read), so the kernel is a latency-hiding stream: a block owns 256 consecutive pixels and NB = 64
// output columns; each of its 4 waves (64 pixels) runs on its own -- no LDS, no barrier -- loading its activation
// AND weight fragments straight from global memory into MFMA operand registers (the A-stationary kernel's
// fragment order, conv3x3.hip conv1x1_areg_kernel) through a register ring of D 32-deep k-steps (one wave per
// SIMD, up to 512 VGPRs): D - 1 steps (up to 56 KB per wave) are in flight while one is consumed.  A first
// version with one chunk in flight and the weights double-buffered in LDS behind a barrier per chunk was
// latency-bound (2.4 us per chunk; ResNet-50 stage-4 conv3 data gradient 76 us against a 14 us floor,
// gpurun_out/r4_02).  The N / 64 column tiles of a pixel tile are consecutive in the XCD-aware block order, so
// they run together on one XCD and the activation / weight re-reads are served by its L2: HBM sees x about once.
//
// PRE operand prologues (BatchNorm backward apply of the layer whose gradient is x, fused into the loads;
// dt also written to pre_out by column tile 0 for the weight gradient):
//   PRE_GM   x = gm (already ReLU-masked): dt = k*gm + A*t + B            (bn_bwd_apply mode 0)
//   PRE_MASK x = the block output's gradient g, masked by the ReLU bits pre_mask ([P][K/8] bytes, bit c&7 of
//            byte c>>3; bn_apply's want_mask): dt = k*(g*bit) + A*t + B   (bn_bwd_apply mode 3)
// The second form is the Bottleneck's conv3 data gradient reading the block output's gradient directly: the
// separate BN3 apply pass (read g and t3, write dt3, then read dt3 again here) disappears.
// Epilogues: conv_direct.h c3_epilogue (plain / residual (masked) / BN statistics / fused BN backward).
// Reference layers: pytorch_code/model_ops/resnet.py:44-64 (Bottleneck conv1 / conv3).
#include "conv_direct.h"

namespace {
using namespace pg;

enum { PRE_NONE = 0, PRE_GM = 1, PRE_MASK = 3 };
constexpr int W1_NB = 64;

template <int EPI, int PRE>
__global__ void __launch_bounds__(256, 1) conv1x1_wide_kernel(C3Args a) {
    constexpr int NB = W1_NB, FN = NB / 16;
    // register ring of D 32-deep k-steps (D - 1 in flight while one is consumed; one wave per SIMD, <= 512 VGPRs,
    // <= 63 loads outstanding): plain 8 loads per step, D = 8 (56 KB in flight per wave); PRE 16 loads, D = 4
    constexpr int D = PRE == PRE_NONE ? 8 : 4;
    extern __shared__ __attribute__((aligned(16))) float coef[];               // PRE: [3][K] k, A, B
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int groups = a.ntiles;
    const int t = xcd_remap(blockIdx.x, a.tiles * groups);
    const int tile = t / groups, nt = t - tile * groups;
    const int p0 = tile * C3_BM, n0 = nt * NB;
    const int K = a.C, KS = K >> 5;                      // 32-deep k-steps

    // this lane's 4 pixels (one per 16-row fragment); rows past P read row P-1 (never stored or counted)
    bool pv[4];
    long prow[4];
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
        const int p = p0 + wave * 64 + fm * 16 + (lane & 15);
        pv[fm] = p < a.P;
        prow[fm] = (long)(pv[fm] ? p : a.P - 1) * K;
    }
    const int lk = (lane >> 4) * 8;                      // this lane's 8 channels within a 32-deep k-step
    const bf16_t* wrow[FN];                              // weight fragment rows of this lane (W^T [N][K], K-major)
#pragma unroll
    for (int f = 0; f < FN; ++f) wrow[f] = a.w + (long)(n0 + f * 16 + (lane & 15)) * K + lk;

    // the ring: activation and weight fragments of D k-steps, [slot][fm | fn] (+ t and mask word for PRE).
    // Loads are unconditional (a step past the end re-reads the last one) so the wait counts stay static.
    u16x8_t xr[D][4], br[D][FN], tr[PRE ? D : 1][4];
    uint32_t mr[PRE == PRE_MASK ? D : 1][4];
    auto load = [&](auto SL, int ks) {
        constexpr int sl = decltype(SL)::value;
        const int k = (ks < KS ? ks : KS - 1) * 32;
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            xr[sl][fm] = *reinterpret_cast<const u16x8_t*>(a.x + prow[fm] + k + lk);
            if constexpr (PRE != PRE_NONE) tr[sl][fm] = *reinterpret_cast<const u16x8_t*>(a.pre_t + prow[fm] + k + lk);
        }
#pragma unroll
        for (int f = 0; f < FN; ++f) br[sl][f] = *reinterpret_cast<const u16x8_t*>(wrow[f] + k);
        if constexpr (PRE == PRE_MASK) {
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)          // 4 mask bytes = the step's 32 channels of the pixel
                mr[sl][fm] = *reinterpret_cast<const uint32_t*>(a.pre_mask + ((prow[fm] + k) >> 3));
        }
    };

    static_for<0, D - 1>([&](auto S) { load(S, (int)decltype(S)::value); });      // steps 0 .. D-2 in flight
    if constexpr (PRE != PRE_NONE) {
        // BatchNorm-backward coefficients of all K channels, once per block (under the first loads)
        const float invL = (float)(1.0 / (double)a.P);
        for (int c = tid; c < K; c += 256) {
            const float is = a.pre_invstd[c], kk = (a.pre_gamma ? a.pre_gamma[c] : 1.f) * is;
            const float dg = a.pre_dgamma[c] * invL, db = a.pre_dbeta[c] * invL;
            coef[c] = kk;
            coef[K + c] = -kk * is * dg;
            coef[2 * K + c] = kk * (a.pre_mean[c] * is * dg - db);
        }
        __syncthreads();
    }

    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // the dt stores are unconditional inside the loop (a divergent store makes the wait counts path-dependent and
    // the compiler then drains the ring): two copies of the loop, with and without them; rows past P store row
    // P-1's dt, which its owning lane stores too (same bytes)
    auto run = [&](auto WDT) {
    constexpr bool write_dt = decltype(WDT)::value;
    for (int k0 = 0; k0 < KS; k0 += D) {
        static_for<0, D>([&](auto S) {
            constexpr int s = decltype(S)::value;
            const int ks = k0 + s;
            // step ks + D - 1 into the slot step ks - 1 has left: D - 1 steps stay in flight
            load(std::integral_constant<int, (s + D - 1) % D>{}, ks + D - 1);
            if (ks < KS) {
                bf16x8_t af[4];
                if constexpr (PRE == PRE_NONE) {
#pragma unroll
                    for (int fm = 0; fm < 4; ++fm) af[fm] = __builtin_bit_cast(bf16x8_t, xr[s][fm]);
                } else {
                    const int c = ks * 32 + lk;
                    PreCoef pc;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        pc.k[j] = coef[c + j];
                        pc.A[j] = coef[K + c + j];
                        pc.B[j] = coef[2 * K + c + j];
                    }
#pragma unroll
                    for (int fm = 0; fm < 4; ++fm) {
                        u16x8_t g = xr[s][fm];
                        if constexpr (PRE == PRE_MASK) {
                            const uint32_t bits = (mr[s][fm] >> (8 * (lane >> 4))) & 0xFFu;    // 8 channel bits
#pragma unroll
                            for (int j = 0; j < 8; ++j) g[j] = ((bits >> j) & 1u) ? g[j] : (unsigned short)0;
                        }
                        const u16x8_t d = pre_apply(pc, g, tr[s][fm]);
                        if constexpr (write_dt) *reinterpret_cast<u16x8_t*>(a.pre_out + prow[fm] + c) = d;
                        af[fm] = __builtin_bit_cast(bf16x8_t, d);
                    }
                }
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            __builtin_bit_cast(bf16x8_t, br[s][fn]), af[fm], acc[fm][fn], 0, 0, 0);
            }
        });
    }
    };
    if (PRE != PRE_NONE && a.pre_out != nullptr && nt == 0) run(std::true_type{});
    else run(std::false_type{});
    c3_epilogue<NB, EPI>(a, acc, tile, p0, n0, wave, lane, pv);
}

template <int EPI, int PRE>
int wide_launch(const C3Args& a, hipStream_t st) {
    const int sm = PRE != PRE_NONE ? 3 * a.C * 4 : 0;
    hipLaunchKernelGGL((conv1x1_wide_kernel<EPI, PRE>), dim3(a.tiles * a.ntiles), dim3(256), sm, st, a);
    PDNN_LAUNCH_RET;
}

template <int PRE>
int wide_dispatch(const C3Args& a, int epi, hipStream_t st) {
    switch (epi) {
        case C3_BNB: return wide_launch<C3_BNB, PRE>(a, st);
        case C3_STATS: return wide_launch<C3_STATS, PRE>(a, st);
        case C3_RES: return wide_launch<C3_RES, PRE>(a, st);
        default: return wide_launch<C3_PLAIN, PRE>(a, st);
    }
}

}  // namespace

static FastDiv w1_fdiv(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}

// Shapes the long-reduction kernel takes: K a multiple of 64 from 512 (the coefficient table of the PRE forms
// stays small), N % 64 == 0.
PDNN_API int pdnn_conv1x1_wide_supported(long P, int K, int N) {
    return K >= 512 && K <= 8192 && K % 64 == 0 && N % W1_NB == 0 && N >= W1_NB && P > 0 &&
           P * (long)K < (1L << 31) ? 1 : 0;
}

// y[P][N] = x[P][K] . w[N][K]^T for K >= 512.  Epilogue / operand arguments as pdnn_conv1x1_panel (slab rows:
// pdnn_conv1x1_panel_stats_rows); pre_mask (with pre_t): the PRE_MASK prologue (x = the masked gradient's
// source, bn_bwd_apply mode 3), else with pre_t the PRE_GM one (mode 0).
PDNN_API int pdnn_conv1x1_wide(const bf16_t* x, const bf16_t* w, bf16_t* y, long P, int K, int N, float* stats,
                               const bf16_t* res, const uint8_t* res_mask, const bf16_t* bn_x, const float* bn_mean,
                               const float* bn_invstd, const float* bn_mscale, const float* bn_mshift,
                               const bf16_t* pre_t, const float* pre_mean,
                               const float* pre_invstd, const float* pre_gamma, const float* pre_dgamma,
                               const float* pre_dbeta, bf16_t* pre_out, const uint8_t* pre_mask, hipStream_t st) {
    if (!pdnn_conv1x1_wide_supported(P, K, N) || (bn_x && !stats) || (res_mask && !res)) return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y; a.C = K; a.N = N; a.P = (int)P;
    a.dW = w1_fdiv(1); a.dH = w1_fdiv(1);
    a.stats = stats; a.res = res; a.rmask = res_mask;
    a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
    a.pre_t = pre_t; a.pre_mean = pre_mean; a.pre_invstd = pre_invstd; a.pre_gamma = pre_gamma;
    a.pre_dgamma = pre_dgamma; a.pre_dbeta = pre_dbeta; a.pre_out = pre_out; a.pre_mask = pre_mask;
    if (pre_t && !(pre_mean && pre_invstd && pre_dgamma && pre_dbeta)) return (int)hipErrorInvalidValue;
    if ((pre_out || pre_mask) && !pre_t) return (int)hipErrorInvalidValue;
    if (bn_x && !(bn_mean && bn_invstd && bn_mscale && bn_mshift)) return (int)hipErrorInvalidValue;
    const int epi = bn_x ? C3_BNB : (stats ? C3_STATS : (res ? C3_RES : C3_PLAIN));
    a.tiles = (int)cdiv(P, C3_BM);
    a.ntiles = N / W1_NB;
    if (pre_mask) return wide_dispatch<PRE_MASK>(a, epi, st);
    if (pre_t) return wide_dispatch<PRE_GM>(a, epi, st);
    return wide_dispatch<PRE_NONE>(a, epi, st);
}
