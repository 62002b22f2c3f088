// Direct 3x3 / stride-1 / pad-1 convolution on MFMA with an LDS-resident input halo (gfx950).
//
// The generic implicit-GEMM engine (gemm_mfma.hip) gathers the A operand of a 3x3 conv from global
// memory once per tap: every input element is fetched 9 times through L1/L2, and the 128-row tiles
// spend their K-steps waiting on those gathers (r3 PMC: the stage-1 3x3 data gradient ran at 9% of the
// bf16 peak, 2-3x its HBM floor; profiles/resnet50_bs256_pmc_r3_before.txt).
//
// Here a block owns BM = 256 consecutive output pixels (row-major over the whole batch, so tiles may
// straddle image boundaries) and NB = 64 / 128 output channels.  Per 64-channel input chunk it stages
// the HALO of its pixels -- the full-width input rows from one above its first row to one below its
// last, a CONTIGUOUS range of NHWC memory -- into LDS once (each input byte is read ~1.1-1.9x instead
// of 9x), then runs the 9 taps as shifted LDS reads: the A fragment of tap (r, s) for output pixel
// (y, x) is halo pixel (y + r - 1, x + s - 1).  Taps that fall outside the image (padding, or the
// neighbouring image of a straddling tile) are redirected to an all-zero pixel at the end of the halo,
// so there is no per-element predication in the MFMA loop.  The weights of one tap ([NB][64] bf16)
// are double-buffered through LDS, the next tap's fetched into registers under the current tap's MFMAs.
//
// One kernel serves the forward (B = W[K][3][3][C]) and the data gradient (B = the tap-flipped,
// transposed weight W'[C][3][3][K], built by conv3x3_flip_kernel): dx = conv3x3(dy, W').
// Epilogues (same semantics and slab layout as the GEMM engine's, gemm_mfma.hip):
//   C3_PLAIN  y = acc                       C3_RES  y = acc + res
//   C3_STATS  y = acc, per-column partial (sum, sum of squares) of the bf16-rounded outputs
//   C3_BNB    gm = acc * [t*mscale + mshift > 0]  (ReLU mask of the BN that produced t, recomputed),
//             store gm, partial sums of gm and gm * (t - mean) * invstd  (BatchNorm backward)
// one slab row pair per (tile, wave): pdnn_conv3x3_stats_rows().
//
// MFMA: v_mfma_f32_16x16x32_bf16 with swapped operands (weight fragment first), so each lane ends
// with 4 consecutive output channels of one pixel; 4 waves each own 64 pixels x NB channels.
// Reference layers: pytorch_code/model_ops/resnet.py:19-21,44-48 (every 3x3 conv of the ResNets).
#include "conv_direct.h"

namespace {
using namespace pg;

typedef __attribute__((ext_vector_type(8))) int c3v8i;
typedef __attribute__((ext_vector_type(4))) int c3v4i;
constexpr int C3_AMAX_PARTS = 1024;              // fp8.hip FP8_AMAX_PARTS
#ifndef C3_PRE_J
#define C3_PRE_J 3
#endif
#ifndef C3_F8_PRE_J
#define C3_F8_PRE_J 2
#endif

// 16 floats -> 16 fp8 bytes (FMT 0: e4m3fn, saturating at 448; 1: e5m2, at 57344)
template <int FMT>
__device__ __forceinline__ uint4 c3_to_fp8(const float* v) {
    constexpr float MX = FMT ? 57344.f : 448.f;
    int w[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const float c0 = fminf(fmaxf(v[4 * d], -MX), MX), c1 = fminf(fmaxf(v[4 * d + 1], -MX), MX);
        const float c2 = fminf(fmaxf(v[4 * d + 2], -MX), MX), c3 = fminf(fmaxf(v[4 * d + 3], -MX), MX);
        int x = 0;
        if constexpr (FMT) {
            x = __builtin_amdgcn_cvt_pk_bf8_f32(c0, c1, x, false);
            x = __builtin_amdgcn_cvt_pk_bf8_f32(c2, c3, x, true);
        } else {
            x = __builtin_amdgcn_cvt_pk_fp8_f32(c0, c1, x, false);
            x = __builtin_amdgcn_cvt_pk_fp8_f32(c2, c3, x, true);
        }
        w[d] = x;
    }
    return make_uint4((uint32_t)w[0], (uint32_t)w[1], (uint32_t)w[2], (uint32_t)w[3]);
}

// F8 = 0: bf16 operands (v_mfma_f32_16x16x32_bf16, 64-channel chunks).
// F8 = 1 / 2: fp8 (the forward's activations in e4m3 / the data gradient's in e5m2; weights e4m3), 128-channel
// chunks on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales): the bf16 input is
// quantised with the tensor's delayed scale WHILE the halo is staged (no separate quantisation pass, no fp8
// copy in HBM), so a halo pixel is the same 128 bytes and the per-tap work covers twice the channels at the
// same LDS traffic and MFMA cycles.  The staged values' |max| feeds the next call's scale (f8_amax partials).
// FP: the forward prologue relu(x * pro_sc + pro_sh) on the staged operand (its coefficients in LDS like PRE's).
template <int NB, int EPI, bool PRE, int F8 = 0, bool FP = false>
__global__ void __launch_bounds__(256, 2) conv3x3_kernel(C3Args a) {
    constexpr int FN = NB / 16;                  // column fragments per wave (every wave spans all NB)
    constexpr int BCH = NB * 8 / 256;            // 16-byte weight chunks per thread per tap
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const halo = reinterpret_cast<bf16_t*>(smem);
    bf16_t* const bbuf = halo + (a.halo_max + 1) * 64;          // [2][NB][64] K-major, kimg_off swizzle

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int t = xcd_remap(blockIdx.x, a.tiles * a.ntiles);
    const int tile = t / a.ntiles, nt = t - tile * a.ntiles;
    const int p0 = tile * C3_BM, n0 = nt * NB;
    const int plast = min(a.P, p0 + C3_BM) - 1;
    const int gr0 = (int)fdiv((uint32_t)p0, a.dW), gr1 = (int)fdiv((uint32_t)plast, a.dW);
    const int nrows = gr1 - gr0 + 3;
    const int hpx = nrows * a.W;                 // halo pixels of this tile; the zero pixel follows
    const long gp0 = (long)(gr0 - 1) * a.W;      // global pixel of halo pixel 0 (may be negative)

    // this lane's 4 output pixels (one per 16-row fragment): halo base, image coordinates
    int hb[4], py[4], px[4];
    bool pv[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        const int p = p0 + wave * 64 + f * 16 + (lane & 15);
        pv[f] = p < a.P;
        const int pp = pv[f] ? p : plast;
        const int gr = (int)fdiv((uint32_t)pp, a.dW);
        px[f] = pp - gr * a.W;
        py[f] = gr - (int)fdiv((uint32_t)gr, a.dH) * a.H;
        hb[f] = (gr - gr0 + 1) * a.W + px[f];
    }

    [[maybe_unused]] uint32_t tmask[4];         // fp8 path: bit tap of f = tap (r, s) of pixel f inside the image
    if constexpr (F8 != 0) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            uint32_t m = 0;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int dr = tap / 3 - 1, ds = tap % 3 - 1;
                if (pv[f] && (unsigned)(py[f] + dr) < (unsigned)a.H && (unsigned)(px[f] + ds) < (unsigned)a.W) m |= 1u << tap;
            }
            tmask[f] = m;
        }
    }
    // the zero pixel sits after the largest halo (halo_max): taps outside the image read it
    const int zpx = a.halo_max;
    if (tid < 8) *reinterpret_cast<u16x8_t*>(halo + zpx * 64 + tid * 8) = c3_zero8();

    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int nchunks = F8 ? a.C >> 7 : a.C >> 6;
    const long wrow = 9L * a.C;                   // elements per weight row n
    u16x8_t rb[BCH];
    [[maybe_unused]] const uint8_t* wb8 =
        reinterpret_cast<const uint8_t*>(a.w) + (long)(n0 + (tid >> 3)) * wrow + (tid & 7) * 16;
    auto load_b = [&](int c0, int tap) {
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int li = tid + 256 * i, row = li >> 3, q = li & 7;
            if constexpr (F8 != 0)   // rows tid / 8 + 32 i: one base, uniform offsets
                rb[i] = *reinterpret_cast<const u16x8_t*>(wb8 + (long)(32 * i) * wrow + (long)tap * a.C + c0);
            else
                rb[i] = *reinterpret_cast<const u16x8_t*>(a.w + (long)(n0 + row) * wrow + (long)tap * a.C + c0 + q * 8);
        }
    };
    auto store_b = [&](int buf) {
        bf16_t* B = bbuf + buf * NB * 64;
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int li = tid + 256 * i, row = li >> 3, q = li & 7;
            *reinterpret_cast<u16x8_t*>(B + kimg_off(row, q)) = rb[i];
        }
    };

    [[maybe_unused]] float qs = 0.f, amx = 0.f;
    if constexpr (F8 != 0) qs = a.f8_scale[0];

    for (int ck = 0; ck < nchunks; ++ck) {
        const int c0 = F8 ? ck << 7 : ck << 6;
        if (ck) __syncthreads();                 // the previous chunk's halo / weights are no longer read
        const int nch = hpx * 8;
        if constexpr (F8 != 0) {
            // ---- stage the fp8 halo of this 128-channel chunk: 16 channels (32 bf16 bytes -> 16 fp8 bytes) per
            // 16-byte chunk i & 7 of halo pixel i >> 3
            // PRE: the chunk's BN-backward coefficients in LDS (weight buffer 1: idle until tap 0's store)
            constexpr int J = PRE ? C3_F8_PRE_J : 4;
            [[maybe_unused]] float* coef = reinterpret_cast<float*>(bbuf + NB * 64);
            if constexpr (PRE) {
                pre_coef_lds<128>(a, c0, coef, tid);
                __syncthreads();
            } else if constexpr (FP) {
                fpro_coef_lds<128>(a, c0, coef, tid);
                __syncthreads();
            }
            for (int i0 = 0; i0 < nch; i0 += 256 * J) {
                u16x8_t v[J][2], tv[PRE ? J : 1][2];
                bool okj[J];
                int gpj[J];
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int i = i0 + j * 256 + tid;
                    const long gp = gp0 + (i >> 3);
                    okj[j] = i < nch && gp >= 0 && gp < a.P;
                    const long gc = gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp);
                    gpj[j] = (int)gc;
                    const bf16_t* src = a.x + gc * a.C + c0 + (i & 7) * 16;
                    v[j][0] = *reinterpret_cast<const u16x8_t*>(src);
                    v[j][1] = *reinterpret_cast<const u16x8_t*>(src + 8);
                    if constexpr (PRE) {
                        const bf16_t* ts = a.pre_t + gc * a.C + c0 + (i & 7) * 16;
                        tv[j][0] = *reinterpret_cast<const u16x8_t*>(ts);
                        tv[j][1] = *reinterpret_cast<const u16x8_t*>(ts + 8);
                    }
                }
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    if constexpr (PRE) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            v[j][h] = pre_apply_lds<128>(coef, (tid & 7) * 16 + 8 * h, v[j][h], tv[j][h]);
                            if (a.pre_out && nt == 0 && okj[j] && gpj[j] >= p0 && gpj[j] <= plast)
                                *reinterpret_cast<u16x8_t*>(a.pre_out + (long)gpj[j] * a.C + c0 + (tid & 7) * 16 + 8 * h) =
                                    v[j][h];
                        }
                    }
                    if constexpr (FP) {
                        v[j][0] = fpro_apply_lds<128>(coef, (tid & 7) * 16, v[j][0]);
                        v[j][1] = fpro_apply_lds<128>(coef, (tid & 7) * 16 + 8, v[j][1]);
                    }
                    float f[16];
                    unpack8(v[j][0], f);
                    unpack8(v[j][1], f + 8);
                    float m = 0.f;
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        m = fmaxf(m, fabsf(f[e]));
                        f[e] *= qs;
                    }
                    if (okj[j]) amx = fmaxf(amx, m);
                    const uint4 q8 = c3_to_fp8<F8 - 1>(f);
                    const int i = i0 + j * 256 + tid;
                    const int off = i < nch ? halo_off(i >> 3, i & 7) : zpx * 64 + (i & 7) * 8;
                    *reinterpret_cast<u16x8_t*>(halo + off) = mask16(__builtin_bit_cast(u16x8_t, q8), okj[j]);
                }
            }
            load_b(c0, 0);
            store_b(0);
            __syncthreads();
            const int g = lane >> 4;
#pragma unroll 1
            for (int tap = 0; tap < 9; ++tap) {
                const int dr = tap / 3 - 1, ds = tap - (tap / 3) * 3 - 1;
                // branch-free tap body (tap 8 re-fetches its own weights into the idle buffer): with a conditional
                // store the MFMAs were sunk below it, every fragment was live at once and the kernel spilled
                load_b(c0, tap < 8 ? tap + 1 : 8);
                const bf16_t* B = bbuf + (tap & 1) * NB * 64;
                c3v8i bq[FN];
#pragma unroll
                for (int f = 0; f < FN; ++f) {
                    const int row = f * 16 + (lane & 15);
                    const c3v4i lo = *reinterpret_cast<const c3v4i*>(B + kimg_off(row, 2 * g));
                    const c3v4i hi = *reinterpret_cast<const c3v4i*>(B + kimg_off(row, 2 * g + 1));
                    bq[f] = c3v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
                // one pixel fragment at a time against all NB weight columns (the 4 x FN accumulators, the FN weight
                // fragments and the 9-tap state leave no room for all four pixel fragments at once)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) {
                    const bool v = (tmask[fm] >> tap) & 1;
                    const int hp = v ? hb[fm] + dr * a.W + ds : zpx;
                    const c3v4i lo = *reinterpret_cast<const c3v4i*>(halo + halo_off(hp, 2 * g));
                    const c3v4i hi = *reinterpret_cast<const c3v4i*>(halo + halo_off(hp, 2 * g + 1));
                    const c3v8i af = c3v8i{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                            bq[fn], af, acc[fm][fn], 0, F8 - 1, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
                }
                store_b((tap + 1) & 1);
                __syncthreads();
            }
            continue;
        }
        // ---- stage the halo of this 64-channel chunk: contiguous pixels gp0 .. gp0 + hpx - 1
        // PRE: two operands live per load; the chunk's BN-backward coefficients in LDS (weight buffer 1, idle
        // until tap 0's store), not 24 VGPRs, so more loads stay in flight
        constexpr int J = PRE ? (NB == 128 ? C3_PRE_J : 4) : 8;
        [[maybe_unused]] float* coef = reinterpret_cast<float*>(bbuf + NB * 64);
        if constexpr (PRE) {
            pre_coef_lds<64>(a, c0, coef, tid);
            __syncthreads();
        } else if constexpr (FP) {
            fpro_coef_lds<64>(a, c0, coef, tid);
            __syncthreads();
        }
        for (int i0 = 0; i0 < nch; i0 += 256 * J) {
            u16x8_t v[J], tv[PRE ? J : 1];
            bool okj[J];
            int gpj[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                // load unconditionally from a clamped (valid) address, then select: a conditional load
                // makes hipcc branch around every element and drain vmcnt each time
                const int i = i0 + j * 256 + tid;
                const long gp = gp0 + (i >> 3);
                okj[j] = i < nch && gp >= 0 && gp < a.P;
                const long gc = gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp);
                gpj[j] = (int)gc;
                v[j] = *reinterpret_cast<const u16x8_t*>(a.x + gc * a.C + c0 + (i & 7) * 8);
                if constexpr (PRE) tv[j] = *reinterpret_cast<const u16x8_t*>(a.pre_t + gc * a.C + c0 + (i & 7) * 8);
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                if constexpr (PRE) {
                    v[j] = pre_apply_lds<64>(coef, (tid & 7) * 8, v[j], tv[j]);
                    // own pixels (each written by exactly one block: column tile 0 of its pixel tile)
                    if (a.pre_out && nt == 0 && okj[j] && gpj[j] >= p0 && gpj[j] <= plast)
                        *reinterpret_cast<u16x8_t*>(a.pre_out + (long)gpj[j] * a.C + c0 + (tid & 7) * 8) = v[j];
                }
                if constexpr (FP) v[j] = fpro_apply_lds<64>(coef, (tid & 7) * 8, v[j]);
                v[j] = mask16(v[j], okj[j]);     // masked, not selected: keeps the load unconditional
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                // past the halo: the (zero) value goes to the zero pixel, so the store needs no branch either
                const int i = i0 + j * 256 + tid;
                const int off = i < nch ? halo_off(i >> 3, i & 7) : zpx * 64 + (i & 7) * 8;
                *reinterpret_cast<u16x8_t*>(halo + off) = v[j];
            }
        }
        load_b(c0, 0);
        store_b(0);
        __syncthreads();
#pragma unroll 1
        for (int tap = 0; tap < 9; ++tap) {
            const int dr = tap / 3 - 1, ds = tap - (tap / 3) * 3 - 1;
            if (tap < 8) load_b(c0, tap + 1);                    // next tap's weights under this tap's MFMAs
            int hp[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const bool v = pv[f] && (unsigned)(py[f] + dr) < (unsigned)a.H && (unsigned)(px[f] + ds) < (unsigned)a.W;
                hp[f] = v ? hb[f] + dr * a.W + ds : zpx;
            }
            const bf16_t* B = bbuf + (tap & 1) * NB * 64;
            // one 32-deep k-step at a time: both in flight would hold 2x the fragments (spills at NB = 128)
#pragma unroll 1
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8_t af[4], bfr[FN];
                const int q = ks * 4 + (lane >> 4);
#pragma unroll
                for (int f = 0; f < 4; ++f)
                    af[f] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(halo + halo_off(hp[f], q)));
#pragma unroll
                for (int f = 0; f < FN; ++f) bfr[f] = frag_kmajor(B, f * 16 + (lane & 15), ks, lane);
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af[fm], acc[fm][fn], 0, 0, 0);
            }
            if (tap < 8) {
                store_b((tap + 1) & 1);
                __syncthreads();
            }
        }
    }

    if constexpr (F8 != 0) {
        amx = wave_max(amx);
        if (lane == 0)
            atomicMax(reinterpret_cast<unsigned int*>(a.f8_amax + (blockIdx.x & (C3_AMAX_PARTS - 1))), __float_as_uint(amx));
        const float gs = a.f8_inv[0] * a.f8_winv[0];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[i][j][e] *= gs;
    }
    c3_epilogue<NB, EPI>(a, acc, tile, p0, n0, wave, lane, pv);
}

// C = N = 64 (ResNet stage 1): all 9 taps of the weight stay resident in LDS (72 KB), one persistent
// block per CU loops over pixel tiles, and the NEXT tile's halo is fetched into registers while the
// current tile computes (cdna_hip_programming.md T14: issue early, write to LDS after the barrier).  No
// barrier inside the 9-tap MFMA sequence; two per tile.
constexpr int C3R_HREG = 16;                     // halo chunks per thread in flight (halo <= 512 pixels)

template <int EPI>
__global__ void __launch_bounds__(256, 1) conv3x3_w64_kernel(C3Args a) {
    constexpr int NB = 64, FN = 4;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const halo = reinterpret_cast<bf16_t*>(smem);
    bf16_t* const wres = halo + (a.halo_max + 1) * 64;       // [9][64 n][64 k], kimg_off per tap image
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int zpx = a.halo_max;

    // resident weights: 9 * 64 rows * 8 chunks
    for (int i = tid; i < 9 * 64 * 8; i += 256) {
        const int tap = i / 512, row = (i >> 3) & 63, q = i & 7;
        *reinterpret_cast<u16x8_t*>(wres + tap * 4096 + kimg_off(row, q)) =
            *reinterpret_cast<const u16x8_t*>(a.w + (long)row * 576 + tap * 64 + q * 8);
    }
    if (tid < 8) *reinterpret_cast<u16x8_t*>(halo + zpx * 64 + tid * 8) = c3_zero8();

    u16x8_t hreg[C3R_HREG];
    auto tile_geom = [&](int tile, int& gr0, int& nch, long& gp0) {
        const int p0 = tile * C3_BM;
        const int plast = min(a.P, p0 + C3_BM) - 1;
        gr0 = (int)fdiv((uint32_t)p0, a.dW);
        const int gr1 = (int)fdiv((uint32_t)plast, a.dW);
        nch = (gr1 - gr0 + 3) * a.W * 8;
        gp0 = (long)(gr0 - 1) * a.W;
    };
    auto fetch = [&](int tile) {                 // halo chunks -> registers (masked, unconditional loads)
        int gr0, nch;
        long gp0;
        tile_geom(tile, gr0, nch, gp0);
#pragma unroll
        for (int j = 0; j < C3R_HREG; ++j) {
            const int i = j * 256 + tid;
            const long gp = gp0 + (i >> 3);
            const bool ok = i < nch && gp >= 0 && gp < a.P;
            const long gc = gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp);
            const u16x8_t ld = *reinterpret_cast<const u16x8_t*>(a.x + gc * 64 + (i & 7) * 8);
            hreg[j] = mask16(ld, ok);
        }
    };
    auto put = [&](int tile) {                   // registers -> LDS halo (past the halo: the zero pixel)
        int gr0, nch;
        long gp0;
        tile_geom(tile, gr0, nch, gp0);
#pragma unroll
        for (int j = 0; j < C3R_HREG; ++j) {
            const int i = j * 256 + tid;
            const int off = i < nch ? halo_off(i >> 3, i & 7) : zpx * 64 + (i & 7) * 8;
            *reinterpret_cast<u16x8_t*>(halo + off) = hreg[j];
        }
    };

    int tile = blockIdx.x;
    if (tile < a.tiles) fetch(tile);
    for (; tile < a.tiles; tile += gridDim.x) {
        __syncthreads();                          // the previous tile's halo is no longer read
        put(tile);
        __syncthreads();
        const int next = tile + gridDim.x;
        if (next < a.tiles) fetch(next);          // lands under this tile's MFMAs

        int gr0, nch;
        long gp0;
        tile_geom(tile, gr0, nch, gp0);
        const int p0 = tile * C3_BM;
        const int plast = min(a.P, p0 + C3_BM) - 1;
        int hb[4], py[4], px[4];
        bool pv[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int p = p0 + wave * 64 + f * 16 + (lane & 15);
            pv[f] = p < a.P;
            const int pp = pv[f] ? p : plast;
            const int gr = (int)fdiv((uint32_t)pp, a.dW);
            px[f] = pp - gr * a.W;
            py[f] = gr - (int)fdiv((uint32_t)gr, a.dH) * a.H;
            hb[f] = (gr - gr0 + 1) * a.W + px[f];
        }
        f32x4_t acc[4][FN];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int dr = tap / 3 - 1, ds = tap % 3 - 1;
            int hp[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const bool v = pv[f] && (unsigned)(py[f] + dr) < (unsigned)a.H && (unsigned)(px[f] + ds) < (unsigned)a.W;
                hp[f] = v ? hb[f] + dr * a.W + ds : zpx;
            }
            const bf16_t* B = wres + tap * 4096;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8_t af[4], bfr[FN];
                const int q = ks * 4 + (lane >> 4);
#pragma unroll
                for (int f = 0; f < 4; ++f)
                    af[f] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(halo + halo_off(hp[f], q)));
#pragma unroll
                for (int f = 0; f < FN; ++f) bfr[f] = frag_kmajor(B, f * 16 + (lane & 15), ks, lane);
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af[fm], acc[fm][fn], 0, 0, 0);
            }
        }
        c3_epilogue<NB, EPI>(a, acc, tile, p0, 0, wave, lane, pv);
    }
}

// ---------------------------------------------------------------------------------------------------
// 1x1 / stride-1 convs with K = 64 * KC <= 256 input channels, A-stationary: each wave holds the MFMA
// fragments of its 64 pixels x all K channels in VGPRs for the whole block (KC = 4: 128 VGPRs), so the
// activations are read once, straight from global memory in fragment order, and never pass through LDS;
// only the weights stream, NB output columns per step, through a double-buffered LDS image (next step's
// weights fetched into registers under this step's MFMAs, one barrier per step).  LDS traffic is then
// one B fragment per 4 MFMAs, the panel kernel's A-from-LDS reads and its 64 KB+ A panel are gone, and
// K = 256 fits (ResNet-50 stage-3 conv3 forward / conv1 data gradient: 50176 x 256 -> 1024).
// PRE: the BatchNorm-backward apply runs on the fragments as they are loaded (once per pixel tile).
// FP: the forward prologue relu(x * pro_sc + pro_sh) likewise (the BN + ReLU of the layer that produced x, e.g. a
// Bottleneck's conv3 reading t2: a2 = relu(bn2(t2)) is never written), bn_apply's formula and rounding.
// ---------------------------------------------------------------------------------------------------
template <int KC, int NB, int EPI, bool PRE, bool FP = false>
__global__ void __launch_bounds__(256, 2) conv1x1_areg_kernel(C3Args a) {
    constexpr int FN = NB / 16, NKS = 2 * KC, K = 64 * KC;
    constexpr int BPT = NB * KC * 8 / 256;               // 16-byte weight pieces per thread per step
    static_assert(BPT >= 1 && NB * KC * 8 % 256 == 0, "weight step must cover the block");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const bbuf = reinterpret_cast<bf16_t*>(smem);     // [2][KC][NB][64] K-major kimg_off images
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int groups = a.ntiles;
    const int t = xcd_remap(blockIdx.x, a.tiles * groups);
    const int tile = t / groups, grp = t - tile * groups;
    const int steps = (a.N / NB) / groups;
    const int c00 = grp * steps;
    const int p0 = tile * C3_BM;

    u16x8_t rb[BPT];
    auto load_b = [&](int s) {
        const int n0 = (c00 + s) * NB;
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            const int li = tid + 256 * i, row = li / (KC * 8), rem = li - row * (KC * 8);
            rb[i] = *reinterpret_cast<const u16x8_t*>(a.w + (long)(n0 + row) * K + rem * 8);
        }
    };
    auto store_b = [&](int buf) {
        bf16_t* B = bbuf + buf * (KC * NB * 64);
#pragma unroll
        for (int i = 0; i < BPT; ++i) {
            const int li = tid + 256 * i, row = li / (KC * 8), rem = li - row * (KC * 8);
            *reinterpret_cast<u16x8_t*>(B + (rem >> 3) * (NB * 64) + kimg_off(row, rem & 7)) = rb[i];
        }
    };
    load_b(0);

    // this wave's activation fragments: pixel (wave*64 + fm*16 + lane&15), channels ks*32 + (lane>>4)*8 .. +8
    bool pv[4];
    long prow[4];
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
        const int p = p0 + wave * 64 + fm * 16 + (lane & 15);
        pv[fm] = p < a.P;
        prow[fm] = (long)(pv[fm] ? p : a.P - 1) * K;
    }
    bf16x8_t af[NKS][4];
    if constexpr (!PRE) {
        [[maybe_unused]] float* coef = reinterpret_cast<float*>(bbuf + 2 * KC * NB * 64);      // FP: [2][K]
        if constexpr (FP) {
            for (int c = tid; c < K; c += 256) {
                coef[c] = a.pro_sc[c];
                coef[K + c] = a.pro_sh[c];
            }
            __syncthreads();
        }
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
                // rows past P hold row P-1's values: their outputs are neither stored nor counted in the statistics
                u16x8_t v = *reinterpret_cast<const u16x8_t*>(a.x + prow[fm] + ks * 32 + (lane >> 4) * 8);
                if constexpr (FP) v = fpro_apply_lds<K>(coef, ks * 32 + (lane >> 4) * 8, v);
                af[ks][fm] = __builtin_bit_cast(bf16x8_t, v);
            }
    } else {
        // BN-backward coefficients of all K channels computed once per block into LDS (after the weight
        // buffers), then the fragments are loaded GB k-steps at a time (gm and t of all of them in flight
        // together) and transformed: per-k-step global coefficient loads serialised the prologue
        float* coef = reinterpret_cast<float*>(bbuf + 2 * KC * NB * 64);      // [3][K]: k, A, B
        {
            const float invL = (float)(1.0 / (double)a.P);
            for (int c = tid; c < K; c += 256) {
                const float is = a.pre_invstd[c], kk = (a.pre_gamma ? a.pre_gamma[c] : 1.f) * is;
                const float dg = a.pre_dgamma[c] * invL, db = a.pre_dbeta[c] * invL;
                coef[c] = kk;
                coef[K + c] = -kk * is * dg;
                coef[2 * K + c] = kk * (a.pre_mean[c] * is * dg - db);
            }
        }
        __syncthreads();
        constexpr int GB = KC == 4 ? 2 : (KC == 2 ? 4 : 2);
#pragma unroll
        for (int g0 = 0; g0 < NKS; g0 += GB) {
            u16x8_t v[GB][4], tv[GB][4];
#pragma unroll
            for (int kk = 0; kk < GB; ++kk)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) {
                    const long off = prow[fm] + (g0 + kk) * 32 + (lane >> 4) * 8;
                    v[kk][fm] = *reinterpret_cast<const u16x8_t*>(a.x + off);
                    tv[kk][fm] = *reinterpret_cast<const u16x8_t*>(a.pre_t + off);
                }
#pragma unroll
            for (int kk = 0; kk < GB; ++kk) {
                const int k = (g0 + kk) * 32 + (lane >> 4) * 8;
                PreCoef pc;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    pc.k[j] = coef[k + j];
                    pc.A[j] = coef[K + k + j];
                    pc.B[j] = coef[2 * K + k + j];
                }
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) {
                    const u16x8_t d = pre_apply(pc, v[kk][fm], tv[kk][fm]);
                    if (a.pre_out && grp == 0 && pv[fm]) *reinterpret_cast<u16x8_t*>(a.pre_out + prow[fm] + k) = d;
                    af[g0 + kk][fm] = __builtin_bit_cast(bf16x8_t, d);
                }
            }
        }
    }
    store_b(0);
    __syncthreads();

    for (int s = 0; s < steps; ++s) {
        const bool more = s + 1 < steps;
        if (more) load_b(s + 1);                 // under this step's MFMAs
        const bf16_t* B = bbuf + (s & 1) * (KC * NB * 64);
        f32x4_t acc[4][FN];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // weight fragments one k-step ahead; the scheduling barrier keeps the compiler from hoisting every
        // k-step's LDS reads to the top (that costs 4 * FN * NKS VGPRs, and spills next to the A fragments)
        bf16x8_t bcur[FN], bnxt[FN];
#pragma unroll
        for (int f = 0; f < FN; ++f) bcur[f] = frag_kmajor(B, f * 16 + (lane & 15), 0, lane);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            if (ks + 1 < NKS) {
#pragma unroll
                for (int f = 0; f < FN; ++f)
                    bnxt[f] = frag_kmajor(B + ((ks + 1) >> 1) * (NB * 64), f * 16 + (lane & 15), (ks + 1) & 1, lane);
            }
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bcur[fn], af[ks][fm], acc[fm][fn], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int f = 0; f < FN; ++f) bcur[f] = bnxt[f];
        }
        // the next weights go to LDS before the epilogue (their buffer was last read in step s-1, closed by
        // that step's barrier): their staging registers are then free during the epilogue, which keeps the
        // K = 256 variants with the fused-BN epilogues out of scratch
        if (more) store_b((s + 1) & 1);
        c3_epilogue<NB, EPI>(a, acc, tile, p0, (c00 + s) * NB, wave, lane, pv);
        if (more) __syncthreads();
    }
}

int c3r_smem(int W);

// W'[c][r][s][k] = W[k][2-r][2-s][c]: the data gradient of a 3x3 / stride-1 / pad-1 conv is that conv
// of dy with the tap-flipped, transposed weight.
__global__ void __launch_bounds__(256) conv3x3_flip_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                                           int K, int C) {
    const long n = 9L * K * C;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const int c = (int)(i % C);
        const long r1 = i / C;
        const int tap = (int)(r1 % 9);
        const int k = (int)(r1 / 9);
        wt[((long)c * 9 + (8 - tap)) * K + k] = w[i];
    }
}

int c3_halo_max(int W) {
    const int rows = (C3_BM - 1 + W - 1) / W + 1 + 2;
    return rows * W;
}

// the e4m3 bytes of W -> W' (same per-tensor scale): the fp8 data gradient's weight
__global__ void __launch_bounds__(256) conv3x3_flip8_kernel(const uint8_t* __restrict__ w, uint8_t* __restrict__ wt,
                                                            int K, int C) {
    const long n = 9L * K * C;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const int k = (int)(i % K);              // W'[c][r][s][k]
        const long r0 = i / K;
        const int tap = (int)(r0 % 9), c = (int)(r0 / 9);
        wt[i] = w[((long)k * 9 + (8 - tap)) * C + c];
    }
}

template <int NB>
int c3_smem(int W) { return (c3_halo_max(W) + 1) * 128 + 2 * NB * 128; }

int c3r_smem(int W) { return (c3_halo_max(W) + 1) * 128 + 9 * 64 * 128; }

template <int EPI>
int c3r_launch(const C3Args& a, hipStream_t st) {
    static int attr_done = 0;
    const int sm = c3r_smem(a.W);
    if (sm > attr_done) {
        (void)hipFuncSetAttribute((const void*)conv3x3_w64_kernel<EPI>, hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        attr_done = sm;
    }
    const int grid = a.tiles < grid_cus() ? a.tiles : grid_cus();     // one persistent block per CU
    hipLaunchKernelGGL((conv3x3_w64_kernel<EPI>), dim3(grid), dim3(256), sm, st, a);
    PDNN_LAUNCH_RET;
}

template <int NB, int EPI, bool PRE, int F8 = 0, bool FP = false>
int c3_launch(const C3Args& a, hipStream_t st) {
    static int attr_done = 0;
    const int sm = c3_smem<NB>(a.W);
    if (sm > attr_done) {
        (void)hipFuncSetAttribute((const void*)conv3x3_kernel<NB, EPI, PRE, F8, FP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        attr_done = sm;
    }
    hipLaunchKernelGGL((conv3x3_kernel<NB, EPI, PRE, F8, FP>), dim3(a.tiles * a.ntiles), dim3(256), sm, st, a);
    PDNN_LAUNCH_RET;
}

template <int NB, bool PRE>
int c3_dispatch(const C3Args& a, int epi, hipStream_t st) {
    switch (epi) {
        case C3_BNB: return c3_launch<NB, C3_BNB, PRE>(a, st);
        case C3_STATS: return c3_launch<NB, C3_STATS, PRE>(a, st);
        case C3_RES: return c3_launch<NB, C3_RES, PRE>(a, st);
        default: return c3_launch<NB, C3_PLAIN, PRE>(a, st);
    }
}

}  // namespace



template <int KC, int NB, int EPI, bool PRE, bool FP = false>
int areg_launch(const C3Args& a, hipStream_t st) {
    constexpr int sm = 2 * KC * NB * 128 + (PRE ? 3 * 64 * KC * 4 : (FP ? 2 * 64 * KC * 4 : 0));
    hipLaunchKernelGGL((conv1x1_areg_kernel<KC, NB, EPI, PRE, FP>), dim3(a.tiles * a.ntiles), dim3(256), sm, st, a);
    PDNN_LAUNCH_RET;
}

template <int KC, int NB, bool PRE>
int areg_dispatch(const C3Args& a, int epi, hipStream_t st) {
    if constexpr (!PRE) {
        if (a.pro_sc) {         // forward prologue: the forward epilogues only
            if (epi == C3_STATS) return areg_launch<KC, NB, C3_STATS, false, true>(a, st);
            if (epi == C3_PLAIN) return areg_launch<KC, NB, C3_PLAIN, false, true>(a, st);
            return (int)hipErrorInvalidValue;
        }
    }
    switch (epi) {
        case C3_BNB: return areg_launch<KC, NB, C3_BNB, PRE>(a, st);
        case C3_STATS: return areg_launch<KC, NB, C3_STATS, PRE>(a, st);
        case C3_RES: return areg_launch<KC, NB, C3_RES, PRE>(a, st);
        default: return areg_launch<KC, NB, C3_PLAIN, PRE>(a, st);
    }
}

// K = 64 / 128 / 256 -> (KC, NB) = (1, 64) / (2, 64) / (4, 32): <= ~190 VGPRs, two blocks per CU
template <bool PRE>
int areg_run(C3Args& a, int K, int epi, hipStream_t st) {
    const int nb = K == 256 ? 32 : 64;
    const int chunks = a.N / nb;
    int g = 1;
    while (g < chunks && (long)a.tiles * g < 512 && chunks % (2 * g) == 0) g *= 2;
    a.ntiles = g;
    if (K == 64) return areg_dispatch<1, 64, PRE>(a, epi, st);
    if (K == 128) return areg_dispatch<2, 64, PRE>(a, epi, st);
    return areg_dispatch<4, 32, PRE>(a, epi, st);
}

// the PRE prologue's operands (all or none; t: [P][C] like x, the rest fp32 [C], gamma optional)
static bool set_pre(C3Args& a, const bf16_t* t, const float* mean, const float* invstd, const float* gamma,
             const float* dgamma, const float* dbeta, bf16_t* out) {
    a.pre_t = t; a.pre_mean = mean; a.pre_invstd = invstd; a.pre_gamma = gamma;
    a.pre_dgamma = dgamma; a.pre_dbeta = dbeta; a.pre_out = out;
    if (!t) return !out;
    return mean && invstd && dgamma && dbeta;
}
static int c3_force() { return pg::tune().conv3x3_force; }

static FastDiv make_fdiv_c3(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}

// Whether the halo kernel takes a 3x3 / stride-1 / pad-1 conv of this shape (channel multiples of 64,
// the halo + weight buffers within 80 KB so two blocks share a CU).
PDNN_API int pdnn_conv3x3_supported(int Nimg, int H, int W, int C, int N) {
    if (C % 64 || N % 64 || C < 64 || N < 64 || W < 1 || H < 1) return 0;
    // narrow images: a 256-pixel tile spans so many rows that the implicit-GEMM engine's 128-row tiles win
    // (ResNet-50 7x7x512, tools/bench_conv3x3.py: 93 / 134 us vs 130 / 152 fwd / dgrad); tuning conv3x3_force
    if (W < 12 && !c3_force()) return 0;
    if ((long)Nimg * H * W >= (1L << 31) / 2) return 0;
    const int nb = N % 128 == 0 ? 128 : 64;
    const int sm = nb == 128 ? c3_smem<128>(W) : c3_smem<64>(W);
    return sm <= 80 * 1024 ? 1 : 0;
}

// 1: take every supported channel shape regardless of the image width (tests); returns the previous
PDNN_API int pdnn_conv3x3_force(int f) {
    const int old = c3_force();
    pg::tune().conv3x3_force = f ? 1 : 0;
    return old;
}

// Slab rows (pairs of sum / sum-of-squares rows) the C3_STATS / C3_BNB epilogues write.
PDNN_API int pdnn_conv3x3_stats_rows(int Nimg, int H, int W) {
    return (int)cdiv((long)Nimg * H * W, C3_BM) * 4;
}

PDNN_API int pdnn_conv3x3_flip_tiled(const bf16_t* w, bf16_t* wt, int K, int C, hipStream_t st);

PDNN_API int pdnn_conv3x3_flip(const bf16_t* w, bf16_t* wt, int K, int C, hipStream_t st) {
    if (K % 8 == 0 && C % 8 == 0) return pdnn_conv3x3_flip_tiled(w, wt, K, C, st);     // elementwise.hip
    hipLaunchKernelGGL(conv3x3_flip_kernel, dim3(stream_grid(9L * K * C, 256)), dim3(256), 0, st, w, wt, K, C);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_conv3x3_flip8(const uint8_t* w, uint8_t* wt, int K, int C, hipStream_t st) {
    hipLaunchKernelGGL(conv3x3_flip8_kernel, dim3(stream_grid(9L * K * C, 256)), dim3(256), 0, st, w, wt, K, C);
    PDNN_LAUNCH_RET;
}

// y[P][N] = conv3x3(x, w) with pad 1, stride 1 (w: [N][3][3][C]); epilogue: stats (fwd BN statistics),
// bn_x (BN-backward mask + sums), res (residual add), else plain.  nb: 0 = automatic, 64 / 128 forced.
// pre_*: optional BN-backward operand prologue (x = gm; the conv's operand is dt = bn_bwd_apply(gm, pre_t),
// also written to pre_out if given): the apply pass of the layer below fused into the loads.
PDNN_API int pdnn_conv3x3(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nimg, int H, int W, int C, int N,
                          float* stats, const bf16_t* res, const uint8_t* res_mask, const bf16_t* bn_x,
                          const float* bn_mean,
                          const float* bn_invstd, const float* bn_mscale, const float* bn_mshift, int nb,
                          const bf16_t* pre_t, const float* pre_mean, const float* pre_invstd,
                          const float* pre_gamma, const float* pre_dgamma, const float* pre_dbeta, bf16_t* pre_out,
                          const float* pro_sc, const float* pro_sh, hipStream_t st) {
    if (!pdnn_conv3x3_supported(Nimg, H, W, C, N)) return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y;
    a.Nimg = Nimg; a.H = H; a.W = W; a.C = C; a.N = N; a.P = Nimg * H * W;
    a.dW = make_fdiv_c3(W); a.dH = make_fdiv_c3(H);
    a.tiles = (int)cdiv(a.P, C3_BM);
    a.halo_max = c3_halo_max(W);
    a.stats = stats; a.res = res; a.rmask = res_mask;
    if (res_mask && !res) return (int)hipErrorInvalidValue;
    if (!set_pre(a, pre_t, pre_mean, pre_invstd, pre_gamma, pre_dgamma, pre_dbeta, pre_out))
        return (int)hipErrorInvalidValue;
    const bool pre = pre_t != nullptr;
    a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
    const int epi = bn_x ? C3_BNB : (stats ? C3_STATS : (res ? C3_RES : C3_PLAIN));
    if (bn_x && !stats) return (int)hipErrorInvalidValue;
    if (!pro_sc != !pro_sh) return (int)hipErrorInvalidValue;
    if (pro_sc) {
        // forward prologue (the BN + ReLU of the layer below): the streaming kernel, statistics or plain epilogue
        if (pre || (epi != C3_STATS && epi != C3_PLAIN)) return (int)hipErrorInvalidValue;
        a.pro_sc = pro_sc; a.pro_sh = pro_sh;
        if (nb <= 1) nb = N % 128 == 0 ? 128 : 64;
        if (nb == 128 && (N % 128 || c3_smem<128>(W) > 80 * 1024)) nb = 64;
        a.ntiles = N / nb;
        if (nb == 128)
            return epi == C3_STATS ? c3_launch<128, C3_STATS, false, 0, true>(a, st) : c3_launch<128, C3_PLAIN, false, 0, true>(a, st);
        return epi == C3_STATS ? c3_launch<64, C3_STATS, false, 0, true>(a, st) : c3_launch<64, C3_PLAIN, false, 0, true>(a, st);
    }
    // 64 -> 64 channels: the weight-resident persistent kernel (nb = 1; measured slower than the streaming
    // kernel at ResNet-50 stage 1, 125 / 173 vs 104 / 142 us fwd / dgrad, gpurun_out/r3_04: one wave per SIMD
    // exposes the LDS latency of the unrolled tap sequence)
    if (nb == 1 && !pre && C == 64 && N == 64 && c3_halo_max(W) * 8 <= C3R_HREG * 256 &&
        c3r_smem(W) <= 160 * 1024) {
        a.ntiles = 1;
        switch (epi) {
            case C3_BNB: return c3r_launch<C3_BNB>(a, st);
            case C3_STATS: return c3r_launch<C3_STATS>(a, st);
            case C3_RES: return c3r_launch<C3_RES>(a, st);
            default: return c3r_launch<C3_PLAIN>(a, st);
        }
    }
    if (nb == 0 || nb == 1) nb = N % 128 == 0 ? 128 : 64;
    if (nb == 128 && (N % 128 || c3_smem<128>(W) > 80 * 1024)) nb = 64;
    a.ntiles = N / nb;
    if (nb == 128) return pre ? c3_dispatch<128, true>(a, epi, st) : c3_dispatch<128, false>(a, epi, st);
    return pre ? c3_dispatch<64, true>(a, epi, st) : c3_dispatch<64, false>(a, epi, st);
}

// Whether the fp8 halo kernel takes this shape: the bf16 kernel's, with 128-channel chunks and 128-wide column tiles.
PDNN_API int pdnn_conv3x3_fp8_supported(int Nimg, int H, int W, int C, int N) {
    return pdnn_conv3x3_supported(Nimg, H, W, C, N) && C % 128 == 0 && N % 128 == 0 &&
           c3_smem<128>(W) <= 80 * 1024;
}

// The fp8 halo conv (conv3x3_kernel F8 = 1 + e5m2): x bf16 [P][C] (quantised while staged with scale[0], the
// staged |max| max-accumulated into amax[FP8_AMAX_PARTS]), wq e4m3 [N][3][3][C] (dequantised by winv[0]), y bf16;
// epilogues plain / stats / fused BN backward (bn_x), pre_*: the BN-backward operand prologue, as pdnn_conv3x3.
// e5m2: the operand in e5m2 (data gradients) instead of e4m3.
PDNN_API int pdnn_conv3x3_fp8(const bf16_t* x, const uint8_t* wq, bf16_t* y, int Nimg, int H, int W, int C, int N,
                              float* stats, const bf16_t* bn_x, const float* bn_mean, const float* bn_invstd,
                              const float* bn_mscale, const float* bn_mshift, const bf16_t* pre_t,
                              const float* pre_mean, const float* pre_invstd, const float* pre_gamma,
                              const float* pre_dgamma, const float* pre_dbeta, bf16_t* pre_out, const float* scale,
                              const float* inv, const float* winv, float* amax, int e5m2, const float* pro_sc,
                              const float* pro_sh, hipStream_t st) {
    if (!pdnn_conv3x3_fp8_supported(Nimg, H, W, C, N) || !scale || !inv || !winv || !amax)
        return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = reinterpret_cast<const bf16_t*>(wq); a.y = y;
    a.Nimg = Nimg; a.H = H; a.W = W; a.C = C; a.N = N; a.P = Nimg * H * W;
    a.dW = make_fdiv_c3(W); a.dH = make_fdiv_c3(H);
    a.tiles = (int)cdiv(a.P, C3_BM);
    a.halo_max = c3_halo_max(W);
    a.stats = stats;
    if (!set_pre(a, pre_t, pre_mean, pre_invstd, pre_gamma, pre_dgamma, pre_dbeta, pre_out))
        return (int)hipErrorInvalidValue;
    a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
    if (bn_x && !stats) return (int)hipErrorInvalidValue;
    a.f8_scale = scale; a.f8_inv = inv; a.f8_winv = winv; a.f8_amax = amax;
    a.ntiles = N / 128;
    const bool pre = pre_t != nullptr;
    if (e5m2) {
        if (bn_x) return pre ? c3_launch<128, C3_BNB, true, 2>(a, st) : c3_launch<128, C3_BNB, false, 2>(a, st);
        if (stats) return (int)hipErrorInvalidValue;
        return pre ? c3_launch<128, C3_PLAIN, true, 2>(a, st) : c3_launch<128, C3_PLAIN, false, 2>(a, st);
    }
    if (pre || bn_x) return (int)hipErrorInvalidValue;
    if (!pro_sc != !pro_sh) return (int)hipErrorInvalidValue;
    if (pro_sc) {
        a.pro_sc = pro_sc; a.pro_sh = pro_sh;
        return stats ? c3_launch<128, C3_STATS, false, 1, true>(a, st) : c3_launch<128, C3_PLAIN, false, 1, true>(a, st);
    }
    return stats ? c3_launch<128, C3_STATS, false, 1>(a, st) : c3_launch<128, C3_PLAIN, false, 1>(a, st);
}

// 1x1 / stride-1 conv on the A-stationary kernel: y[P][N] = x[P][K] . w[N][K]^T, K in {64, 128, 256},
// N % 64 == 0.  Epilogues as pdnn_conv3x3.  Returns hipErrorInvalidValue for shapes it does not take.  (An LDS
// pixel-panel kernel for K <= 128 lost to it: r3_15, 9,844 vs 9,780 img/s; removed in round 4.)
PDNN_API int pdnn_conv1x1_panel_supported(long P, int K, int N) {
    const bool k_ok = K == 64 || K == 128 || K == 256;
    return k_ok && N % 64 == 0 && N >= 64 && P > 0 && P < (1L << 30) ? 1 : 0;
}

PDNN_API int pdnn_conv1x1_panel(const bf16_t* x, const bf16_t* w, bf16_t* y, long P, int K, int N, float* stats,
                                const bf16_t* res, const uint8_t* res_mask, const bf16_t* bn_x, const float* bn_mean,
                                const float* bn_invstd, const float* bn_mscale, const float* bn_mshift,
                                const bf16_t* pre_t, const float* pre_mean, const float* pre_invstd,
                                const float* pre_gamma, const float* pre_dgamma, const float* pre_dbeta,
                                bf16_t* pre_out, const float* pro_sc, const float* pro_sh, hipStream_t st) {
    if (!pdnn_conv1x1_panel_supported(P, K, N) || (bn_x && !stats) || (res_mask && !res) || (!pro_sc != !pro_sh) ||
        (pro_sc && (pre_t || bn_x || res)))
        return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y; a.C = K; a.N = N; a.P = (int)P;
    a.tiles = (int)cdiv(P, C3_BM);
    a.stats = stats; a.res = res; a.rmask = res_mask;
    a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
    if (!set_pre(a, pre_t, pre_mean, pre_invstd, pre_gamma, pre_dgamma, pre_dbeta, pre_out))
        return (int)hipErrorInvalidValue;
    a.pro_sc = pro_sc; a.pro_sh = pro_sh;
    const int epi = bn_x ? C3_BNB : (stats ? C3_STATS : (res ? C3_RES : C3_PLAIN));
    return pre_t ? areg_run<true>(a, K, epi, st) : areg_run<false>(a, K, epi, st);
}

PDNN_API int pdnn_conv1x1_panel_stats_rows(long P) { return (int)cdiv(P, C3_BM) * 4; }
