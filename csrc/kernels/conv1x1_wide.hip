// 1x1 / stride-1 convolutions with a LONG reduction (K = C_in in {512, 1024, 2048}) on MFMA (gfx950):
// y[P][N] = x[P][K] . W[N][K]^T.  In ResNet-50 these are the data gradients of conv3 (dt3 [P][4w] -> [P][w],
// with the BatchNorm-backward epilogue of BN2) in stages 2-4 and of conv1 in stage 4, and the stage-3/4
// forward convs with K >= 512.  On the 128-row implicit-GEMM engine they ran at 9.5-14% of the bf16 peak,
// 2-3x their HBM floor (profiles/resnet50_bs256_pmc_r3_end.txt: 2.95 ms/step).
//
// They are memory-bound (every activation byte feeds 2 * NB flops, NB <= 512 output columns; the HBM
// floor is the x read), so the kernel is a stream: a block owns 256 consecutive pixels and NB = 64 output
// columns; its 4 waves (64 pixels each) load their activation fragments STRAIGHT from global memory into
// MFMA operand registers (the A-stationary kernel's fragment order, conv3x3.hip conv1x1_areg_kernel), one
// 64-deep k-chunk ahead of the MFMAs -- no LDS round trip, 8 KB in flight per wave, 2-3 blocks per CU --
// while the NB x 64 weight slice of each k-chunk is double-buffered through LDS (fetched into registers
// under the previous chunk's MFMAs, one barrier per chunk).  The N / 64 column tiles of a pixel tile are
// consecutive in the XCD-aware block order, so they run together on one XCD and the activation re-reads
// are served by its L2: HBM sees x about once.
//
// PRE operand prologue (BatchNorm backward apply of the layer whose gradient is x, fused into the loads; dt also
// written to pre_out by column tile 0 for the weight gradient): x = gm, dt = k*gm + A*t + B (bn_bwd_apply mode 0).
//
// Where it runs (gpurun_out/r4_02, r4_03, tools/bench_conv1x1.py): the stage-4 conv1 data gradients (K = 512 ->
// N = 1024 / 2048 with the masked residual and the BN1 apply prologue): 81 us against 102 us on the ping-pong
// engine.  It does NOT beat the implicit-GEMM engine on the conv3 data gradients (K >= 512 -> N <= 512 with the
// BN-backward epilogue: 103 / 83 / 76 us vs 99 / 80 / 69 us for stages 2 / 3 / 4) or the K >= 512 forwards, and
// two variants lost outright: folding BN3's backward apply into conv3's data gradient (gout masked by the output
// ReLU bits in the loads, dt3 written here; 217-222 us vs 125-243 us apply + conv) and a version with a per-wave
// register ring 7 k-steps deep and no LDS (one wave per SIMD; 140-190 us: every wave fetching its own weight
// fragments doubled the L1 traffic).
// Epilogues: conv_direct.h c3_epilogue (plain / residual (masked) / BN statistics / fused BN backward).
// Reference layers: pytorch_code/model_ops/resnet.py:44-64 (Bottleneck conv1 / conv3).
#include "conv_direct.h"

namespace {
using namespace pg;

enum { PRE_NONE = 0, PRE_GM = 1 };
constexpr int W1_NB = 64;

template <int EPI, int PRE>
__global__ void __launch_bounds__(256, 2) conv1x1_wide_kernel(C3Args a) {
    constexpr int NB = W1_NB, FN = NB / 16;
    constexpr int BPT = NB * 8 / 256;                    // 16-byte weight pieces per thread per k-chunk
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const bbuf = reinterpret_cast<bf16_t*>(smem);                      // [2][NB][64] kimg images
    float* const coef = reinterpret_cast<float*>(bbuf + 2 * NB * 64);          // PRE: [3][K] k, A, B
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int groups = a.ntiles;
    const int t = xcd_remap(blockIdx.x, a.tiles * groups);
    const int tile = t / groups, nt = t - tile * groups;
    const int p0 = tile * C3_BM, n0 = nt * NB;
    const int K = a.C, KC = K >> 6;

    u16x8_t rb[BPT];
    auto load_b = [&](int kc) {
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            const int li = tid + 256 * i, row = li >> 3, q = li & 7;
            rb[i] = *reinterpret_cast<const u16x8_t*>(a.w + (long)(n0 + row) * K + kc * 64 + q * 8);
        }
    };
    auto store_b = [&](int buf) {
        bf16_t* B = bbuf + buf * NB * 64;
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            const int li = tid + 256 * i, row = li >> 3, q = li & 7;
            *reinterpret_cast<u16x8_t*>(B + kimg_off(row, q)) = rb[i];
        }
    };

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

    // next chunk's operands in flight: activation fragments [ks][fm] (+ t for PRE)
    u16x8_t xa[2][4], ta[PRE ? 2 : 1][4];
    auto load_a = [&](int kc) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
                const long off = prow[fm] + kc * 64 + ks * 32 + lk;
                xa[ks][fm] = *reinterpret_cast<const u16x8_t*>(a.x + off);
                if constexpr (PRE != PRE_NONE) ta[ks][fm] = *reinterpret_cast<const u16x8_t*>(a.pre_t + off);
            }
    };

    load_b(0);
    load_a(0);
    if constexpr (PRE != PRE_NONE) {
        // BatchNorm-backward coefficients of all K channels, once per block
        const float invL = (float)(1.0 / (double)a.P);
        for (int c = tid; c < K; c += 256) {
            const float is = a.pre_invstd[c], kk = (a.pre_gamma ? a.pre_gamma[c] : 1.f) * is;
            const float dg = a.pre_dgamma[c] * invL, db = a.pre_dbeta[c] * invL;
            coef[c] = kk;
            coef[K + c] = -kk * is * dg;
            coef[2 * K + c] = kk * (a.pre_mean[c] * is * dg - db);
        }
    }
    store_b(0);
    __syncthreads();

    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const bool write_dt = PRE != PRE_NONE && a.pre_out != nullptr && nt == 0;
    for (int kc = 0; kc < KC; ++kc) {
        // this chunk's operand fragments (transformed for PRE), then the next chunk's loads are issued
        bf16x8_t af[2][4];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            if constexpr (PRE == PRE_NONE) {
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) af[ks][fm] = __builtin_bit_cast(bf16x8_t, xa[ks][fm]);
            } else {
                const int c = kc * 64 + ks * 32 + lk;
                PreCoef pc;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    pc.k[j] = coef[c + j];
                    pc.A[j] = coef[K + c + j];
                    pc.B[j] = coef[2 * K + c + j];
                }
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) {
                    const u16x8_t d = pre_apply(pc, xa[ks][fm], ta[ks][fm]);
                    if (write_dt && pv[fm]) *reinterpret_cast<u16x8_t*>(a.pre_out + prow[fm] + c) = d;
                    af[ks][fm] = __builtin_bit_cast(bf16x8_t, d);
                }
            }
        }
        const bool more = kc + 1 < KC;
        if (more) {
            load_a(kc + 1);                  // under this chunk's MFMAs
            load_b(kc + 1);
        }
        const bf16_t* B = bbuf + (kc & 1) * NB * 64;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8_t bfr[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) bfr[f] = frag_kmajor(B, f * 16 + (lane & 15), ks, lane);
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af[ks][fm], acc[fm][fn], 0, 0, 0);
        }
        if (more) {
            store_b((kc + 1) & 1);           // buffer (kc+1)&1 was last read in chunk kc-1, closed by its barrier
            __syncthreads();
        }
    }
    c3_epilogue<NB, EPI>(a, acc, tile, p0, n0, wave, lane, pv);
}

template <int EPI, int PRE>
int wide_launch(const C3Args& a, hipStream_t st) {
    const int sm = 2 * W1_NB * 128 + (PRE != PRE_NONE ? 3 * a.C * 4 : 0);
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
// pdnn_conv1x1_panel_stats_rows); with pre_t the PRE_GM prologue (bn_bwd_apply mode 0).
PDNN_API int pdnn_conv1x1_wide(const bf16_t* x, const bf16_t* w, bf16_t* y, long P, int K, int N, float* stats,
                               const bf16_t* res, const uint8_t* res_mask, const bf16_t* bn_x, const float* bn_mean,
                               const float* bn_invstd, const float* bn_mscale, const float* bn_mshift,
                               const bf16_t* pre_t, const float* pre_mean,
                               const float* pre_invstd, const float* pre_gamma, const float* pre_dgamma,
                               const float* pre_dbeta, bf16_t* pre_out, hipStream_t st) {
    if (!pdnn_conv1x1_wide_supported(P, K, N) || (bn_x && !stats) || (res_mask && !res)) return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y; a.C = K; a.N = N; a.P = (int)P;
    a.dW = w1_fdiv(1); a.dH = w1_fdiv(1);
    a.stats = stats; a.res = res; a.rmask = res_mask;
    a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
    a.pre_t = pre_t; a.pre_mean = pre_mean; a.pre_invstd = pre_invstd; a.pre_gamma = pre_gamma;
    a.pre_dgamma = pre_dgamma; a.pre_dbeta = pre_dbeta; a.pre_out = pre_out;
    if (pre_t && !(pre_mean && pre_invstd && pre_dgamma && pre_dbeta)) return (int)hipErrorInvalidValue;
    if (pre_out && !pre_t) return (int)hipErrorInvalidValue;
    if (bn_x && !(bn_mean && bn_invstd && bn_mscale && bn_mshift)) return (int)hipErrorInvalidValue;
    const int epi = bn_x ? C3_BNB : (stats ? C3_STATS : (res ? C3_RES : C3_PLAIN));
    a.tiles = (int)cdiv(P, C3_BM);
    a.ntiles = N / W1_NB;
    if (pre_t) return wide_dispatch<PRE_GM>(a, epi, st);
    return wide_dispatch<PRE_NONE>(a, epi, st);
}
