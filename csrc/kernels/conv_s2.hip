// Direct 3x3 / stride-2 / pad-1 convolution (forward and data gradient) on MFMA with an LDS halo (gfx950).
//
// The stage-transition Bottlenecks of a ResNet (reference: pytorch_code/model_ops/resnet.py:39-56, stride on the
// 3x3 conv2) ran their stride-2 3x3 convs on the implicit-GEMM engine: the data gradient as four parity-class GEMMs
// whose gathers are VALU-bound (8.8% of the bf16 peak, 1.1-1.2 ms per ResNet-50 step on the critical data-gradient
// chain, profiles/resnet50_bs256_pmc_r5_end.txt), the forward through im2col gathers of a materialised a1.
//
// Both directions are rewritten here as the stride-1 halo kernel's structure (conv3x3.hip) on the HALF-resolution
// pixel grid (n, i, j), i < Ho = H / 2, j < Wo = W / 2, where every tap is a unit shift:
//
//   forward   y[i, j] = sum_{r,s} x[2i + r - 1, 2j + s - 1] W[r, s].  Split x into its four parity planes
//             x_ab[i, j] = x[2i + a, 2j + b]: tap r reads plane row parity a = (r != 1) at row offset -1 (r = 0) or
//             0 (r = 1, 2), likewise s.  The block's reduction loops over (plane, 64-channel chunk); the halo of a
//             chunk is that plane's pixels gathered straight from NHWC x (128-byte pixel chunks, stride 2 -- no
//             space-to-depth copy), and only the plane's taps run: 1 + 2 + 2 + 4 = 9 taps per 4 chunks, the same
//             MFMA work as the dense conv.  The BN + ReLU of the layer below (a1 = relu(bn1(t1))) is applied while
//             staging (FP), so a1 is never materialised.
//   data grad dx[2i + a, 2j + b] = sum over the class-(a, b) taps of dy[i + di, j + dj] W[r, s], r = a + 1 - 2 di
//             (di in {0} for a = 0, {0, 1} for a = 1), likewise s: each output parity class is a 1 / 2 / 2 / 4-tap
//             conv of dy at unit offsets.  A block owns one class (its output column tile sits in that class), so no
//             MFMA runs on the zero taps; the grid issues the 4-tap class first.  The halo is dy's (with the BN2
//             backward apply fused into the staging, PRE, writing dt2 for the weight gradient), the epilogue scatters
//             each class's rows to its dx pixels and applies the BN1-backward mask + sums (C3_BNB) there.
//
// Weights: forward W [K][3][3][C] as is; data gradient the transposed W' [C][3][3][K] of conv3x3_flip (tap 8 - t).
// Tiles: 256 half-resolution pixels x 128 output channels, 4 waves, 2 blocks per CU (<= 80 KB LDS).
#include "conv_direct.h"

namespace {
using namespace pg;

constexpr int S2_NB = 128;
#ifndef S2_J
#define S2_J 4
#endif
#ifndef S2_PRE_J
#define S2_PRE_J 2
#endif

template <bool DG, int EPI, bool PRE, bool FP>
__global__ void __launch_bounds__(256, 2) conv3x3s2_kernel(C3Args a) {
    constexpr int NB = S2_NB, FN = NB / 16;
    constexpr int BCH = NB * 8 / 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const halo = reinterpret_cast<bf16_t*>(smem);
    bf16_t* const bbuf = halo + (a.halo_max + 1) * 64;          // [2][NB][64] K-major, kimg_off swizzle

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.tiles * a.ntiles;
    int cls = 0, local = blockIdx.x;
    if constexpr (DG) {
        // heaviest class first (longest-processing-time order): (1,1) 4 taps, (0,1) and (1,0) 2, (0,0) 1
        const int seg = blockIdx.x / T;
        local = blockIdx.x - seg * T;
        cls = seg == 0 ? 3 : (seg == 3 ? 0 : seg);
    }
    const int t = xcd_remap(local, T);
    const int tile = t / a.ntiles, nt = t - tile * a.ntiles;
    const int ca = cls >> 1, cb = cls & 1;
    const int p0 = tile * C3_BM, n0 = nt * NB;
    const int plast = min(a.P, p0 + C3_BM) - 1;
    const int Wo = a.W;
    const int gr0 = (int)fdiv((uint32_t)p0, a.dW), gr1 = (int)fdiv((uint32_t)plast, a.dW);
    // halo rows: forward gr0 - 1 .. gr1 (taps at row offset -1 / 0), data gradient gr0 .. gr1 + 1 (offset 0 / +1)
    constexpr int RLO = DG ? 0 : 1;
    const int hpx = (gr1 - gr0 + 2) * Wo;
    const long gp0 = (long)(gr0 - RLO) * Wo;

    int hb[4], py[4], px[4];
    bool pv[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        const int p = p0 + wave * 64 + f * 16 + (lane & 15);
        pv[f] = p < a.P;
        const int pp = pv[f] ? p : plast;
        const int gr = (int)fdiv((uint32_t)pp, a.dW);
        px[f] = pp - gr * Wo;
        py[f] = gr - (int)fdiv((uint32_t)gr, a.dH) * a.H;
        hb[f] = (gr - gr0 + RLO) * Wo + px[f];
    }
    const int zpx = a.halo_max;
    if (tid < 8) *reinterpret_cast<u16x8_t*>(halo + zpx * 64 + tid * 8) = c3_zero8();

    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int cch = a.C >> 6;
    const int nchunks = DG ? cch : 4 * cch;
    const long wrow = 9L * a.C;
    u16x8_t rb[BCH];
    auto load_b = [&](int c0, int tw) {
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int li = tid + 256 * i, row = li >> 3, q = li & 7;
            rb[i] = *reinterpret_cast<const u16x8_t*>(a.w + (long)(n0 + row) * wrow + (long)tw * a.C + c0 + q * 8);
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
    // tap k of the chunk -> (row offset, column offset, weight tap index); pa / pb: the parity class (data gradient)
    // or the input plane (forward) -- uniform scalar arithmetic, no per-lane tables
    auto tap_of = [&](int k, int pa, int pb, int& dr, int& ds, int& tw) {
        const int kr = pb ? (k >> 1) : k, ks = pb ? (k & 1) : 0;
        if constexpr (DG) {
            dr = kr;
            ds = ks;
            const int r = pa + 1 - 2 * kr, s = pb + 1 - 2 * ks;
            tw = 8 - (3 * r + s);
        } else {
            const int r = pa ? 2 * kr : 1, s = pb ? 2 * ks : 1;
            dr = r == 0 ? -1 : 0;
            ds = s == 0 ? -1 : 0;
            tw = 3 * r + s;
        }
    };

    for (int ck = 0; ck < nchunks; ++ck) {
        const int plane = DG ? cls : ck / cch;
        const int c0 = (DG ? ck : ck - (ck / cch) * cch) << 6;
        const int pa = plane >> 1, pb = plane & 1;
        const int ntap = (1 + pa) * (1 + pb);
        if (ck) __syncthreads();                 // the previous chunk's halo / weights are no longer read
        const int nch = hpx * 8;
        constexpr int J = (PRE || FP) ? S2_PRE_J : S2_J;
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
            [[maybe_unused]] long srcj[FP ? J : 1];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int i = i0 + j * 256 + tid;
                const long gp = gp0 + (i >> 3);
                okj[j] = i < nch && gp >= 0 && gp < a.P;
                const int gc = (int)(gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp));
                gpj[j] = gc;
                long src = gc;
                if constexpr (!DG) {     // half-resolution pixel (gr, jj) of plane (pa, pb) -> full-resolution x pixel
                    const int gr = (int)fdiv((uint32_t)gc, a.dW);
                    src = (long)(2 * gr + pa) * (2 * Wo) + 2 * (gc - gr * Wo) + pb;
                }
                if constexpr (FP) srcj[j] = src;
                v[j] = *reinterpret_cast<const u16x8_t*>(a.x + src * a.C + c0 + (i & 7) * 8);
                if constexpr (PRE) tv[j] = *reinterpret_cast<const u16x8_t*>(a.pre_t + src * a.C + c0 + (i & 7) * 8);
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                if constexpr (PRE) {
                    v[j] = pre_apply_lds<64>(coef, (tid & 7) * 8, v[j], tv[j]);
                    // own pixels of the class-0 column-tile-0 block (each dy pixel written exactly once)
                    if (a.pre_out && cls == 0 && nt == 0 && okj[j] && gpj[j] >= p0 && gpj[j] <= plast)
                        *reinterpret_cast<u16x8_t*>(a.pre_out + (long)gpj[j] * a.C + c0 + (tid & 7) * 8) = v[j];
                }
                if constexpr (FP) {
                    v[j] = fpro_apply_lds<64>(coef, (tid & 7) * 8, v[j]);
                    // a1 as a by-product (pre_out): the own plane pixels' BN + ReLU values -- every input pixel is one
                    // plane pixel of exactly one tile -- so the weight gradient reads a materialised a1 and no
                    // bn_apply pass runs
                    if (a.pre_out && nt == 0 && okj[j] && gpj[j] >= p0 && gpj[j] <= plast)
                        *reinterpret_cast<u16x8_t*>(a.pre_out + srcj[j] * a.C + c0 + (tid & 7) * 8) = v[j];
                }
                v[j] = mask16(v[j], okj[j]);
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int i = i0 + j * 256 + tid;
                const int off = i < nch ? halo_off(i >> 3, i & 7) : zpx * 64 + (i & 7) * 8;
                *reinterpret_cast<u16x8_t*>(halo + off) = v[j];
            }
        }
        int dr0, ds0, tw0;
        tap_of(0, pa, pb, dr0, ds0, tw0);
        load_b(c0, tw0);
        store_b(0);
        __syncthreads();
#pragma unroll 1
        for (int k = 0; k < ntap; ++k) {
            int dr, ds, tw;
            tap_of(k, pa, pb, dr, ds, tw);
            if (k + 1 < ntap) {
                int dr1, ds1, tw1;
                tap_of(k + 1, pa, pb, dr1, ds1, tw1);
                load_b(c0, tw1);                 // next tap's weights under this tap's MFMAs
            }
            int hp[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                bool v;
                if constexpr (DG) v = pv[f] && py[f] + dr < a.H && px[f] + ds < Wo;
                else v = pv[f] && py[f] + dr >= 0 && px[f] + ds >= 0;
                hp[f] = v ? hb[f] + dr * Wo + ds : zpx;
            }
            const bf16_t* B = bbuf + (k & 1) * NB * 64;
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
            if (k + 1 < ntap) {
                store_b((k + 1) & 1);
                __syncthreads();
            }
        }
    }

    long orow[4];
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
        const int p = p0 + wave * 64 + fm * 16 + (lane & 15);
        if constexpr (DG) {          // class (ca, cb) row of half-resolution pixel (gr, j) -> dx pixel (2 gr + ca, 2 j + cb)
            const int pp = pv[fm] ? p : plast;
            const int gr = (int)fdiv((uint32_t)pp, a.dW);
            orow[fm] = ((long)(2 * gr + ca) * (2 * Wo) + 2 * (pp - gr * Wo) + cb) * a.N;
        } else {
            orow[fm] = (long)p * a.N;
        }
    }
    // statistics rows: the 4 class blocks of a pixel tile add into different bins (tile-major stats index 4 tile + cls)
    c3_epilogue_rows<NB, EPI>(a, acc, DG ? tile * 4 + cls : tile, orow, n0, wave, lane, pv);
}

// Data gradient, class pairs: a block owns 64 output channels of TWO parity classes -- pair 0 = (0,0) + (1,1)
// (1 + 4 taps), pair 1 = (0,1) + (1,0) (2 + 2) -- so each staged dy halo feeds 4-5 taps instead of 1-4 and the two
// kinds of blocks carry nearly equal work; the accumulators (2 classes x 64 pixels x 64 channels per wave) take the
// registers of the single-class 128-wide tile.  Plain / fused-BN-backward epilogues (no operand prologue).
template <int EPI>
__global__ void __launch_bounds__(256, 2) conv3x3s2_dgrad_pair_kernel(C3Args a) {
    constexpr int NB = 64, FN = NB / 16;
    constexpr int BCH = NB * 8 / 256;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const halo = reinterpret_cast<bf16_t*>(smem);
    bf16_t* const bbuf = halo + (a.halo_max + 1) * 64;          // [2][NB][64] K-major, kimg_off swizzle

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.tiles * a.ntiles;
    const int pair = blockIdx.x < T ? 0 : 1;                    // the 5-tap pair first
    const int t = xcd_remap(blockIdx.x - pair * T, T);
    const int tile = t / a.ntiles, nt = t - tile * a.ntiles;
    const int p0 = tile * C3_BM, n0 = nt * NB;
    const int plast = min(a.P, p0 + C3_BM) - 1;
    const int Wo = a.W;
    const int gr0 = (int)fdiv((uint32_t)p0, a.dW), gr1 = (int)fdiv((uint32_t)plast, a.dW);
    const int hpx = (gr1 - gr0 + 2) * Wo;                      // dy rows gr0 .. gr1 + 1
    const long gp0 = (long)gr0 * Wo;
    // the pair's classes (slot 0, slot 1) and their tap counts
    const int cl0 = pair ? 1 : 0, cl1 = pair ? 2 : 3;
    const int nt0 = pair ? 2 : 1, ntot = pair ? 4 : 5;

    int hb[4], py[4], px[4];
    bool pv[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
        const int p = p0 + wave * 64 + f * 16 + (lane & 15);
        pv[f] = p < a.P;
        const int pp = pv[f] ? p : plast;
        const int gr = (int)fdiv((uint32_t)pp, a.dW);
        px[f] = pp - gr * Wo;
        py[f] = gr - (int)fdiv((uint32_t)gr, a.dH) * a.H;
        hb[f] = (gr - gr0) * Wo + px[f];
    }
    const int zpx = a.halo_max;
    if (tid < 8) *reinterpret_cast<u16x8_t*>(halo + zpx * 64 + tid * 8) = c3_zero8();

    f32x4_t acc[2][4][FN];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[c][i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int cch = a.C >> 6;
    const long wrow = 9L * a.C;
    u16x8_t rb[BCH];
    auto load_b = [&](int c0, int tw) {
#pragma unroll
        for (int i = 0; i < BCH; ++i) {
            const int li = tid + 256 * i, row = li >> 3, q = li & 7;
            rb[i] = *reinterpret_cast<const u16x8_t*>(a.w + (long)(n0 + row) * wrow + (long)tw * a.C + c0 + q * 8);
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
    // global tap g of the pair (0 .. ntot-1) -> class slot, (di, dj) offsets, W' tap index
    auto tap_of = [&](int g, int& slot, int& dr, int& ds, int& tw) {
        slot = g >= nt0 ? 1 : 0;
        const int k = g - (slot ? nt0 : 0);
        const int cls = slot ? cl1 : cl0, pa = cls >> 1, pb = cls & 1;
        const int kr = pb ? (k >> 1) : k, kc = pb ? (k & 1) : 0;
        dr = kr;
        ds = kc;
        tw = 8 - (3 * (pa + 1 - 2 * kr) + (pb + 1 - 2 * kc));
    };

    for (int ck = 0; ck < cch; ++ck) {
        const int c0 = ck << 6;
        if (ck) __syncthreads();
        const int nch = hpx * 8;
        constexpr int J = S2_J;
        for (int i0 = 0; i0 < nch; i0 += 256 * J) {
            u16x8_t v[J];
            bool okj[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int i = i0 + j * 256 + tid;
                const long gp = gp0 + (i >> 3);
                okj[j] = i < nch && gp >= 0 && gp < a.P;
                const long gc = gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp);
                v[j] = *reinterpret_cast<const u16x8_t*>(a.x + gc * a.C + c0 + (i & 7) * 8);
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int i = i0 + j * 256 + tid;
                const int off = i < nch ? halo_off(i >> 3, i & 7) : zpx * 64 + (i & 7) * 8;
                *reinterpret_cast<u16x8_t*>(halo + off) = mask16(v[j], okj[j]);
            }
        }
        {
            int sl, dr, ds, tw;
            tap_of(0, sl, dr, ds, tw);
            load_b(c0, tw);
        }
        store_b(0);
        __syncthreads();
        // the class slots one after the other (compile-time accumulator index), the global tap counter g running on
        // through both (weight double buffer parity, next-tap prefetch across the slot boundary)
        static_for<0, 2>([&](auto SL) {
            const int gend = SL ? ntot : nt0;
#pragma unroll 1
            for (int g = SL ? nt0 : 0; g < gend; ++g) {
                int sl, dr, ds, tw;
                tap_of(g, sl, dr, ds, tw);
                if (g + 1 < ntot) {
                    int sl1, dr1, ds1, tw1;
                    tap_of(g + 1, sl1, dr1, ds1, tw1);
                    load_b(c0, tw1);
                }
                int hp[4];
#pragma unroll
                for (int f = 0; f < 4; ++f) {
                    const bool ok = pv[f] && py[f] + dr < a.H && px[f] + ds < Wo;
                    hp[f] = ok ? hb[f] + dr * Wo + ds : zpx;
                }
                const bf16_t* B = bbuf + (g & 1) * NB * 64;
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
                            acc[SL][fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af[fm], acc[SL][fm][fn], 0, 0, 0);
                }
                if (g + 1 < ntot) {
                    store_b((g + 1) & 1);
                    __syncthreads();
                }
            }
        });
    }

    static_for<0, 2>([&](auto SL) {
        const int cls = SL ? cl1 : cl0, ca = cls >> 1, cb = cls & 1;
        long orow[4];
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const int p = p0 + wave * 64 + fm * 16 + (lane & 15);
            const int pp = pv[fm] ? p : plast;
            const int gr = (int)fdiv((uint32_t)pp, a.dW);
            orow[fm] = ((long)(2 * gr + ca) * (2 * Wo) + 2 * (pp - gr * Wo) + cb) * a.N;
        }
        c3_epilogue_rows<NB, EPI>(a, acc[SL], tile * 4 + cls, orow, n0, wave, lane, pv);
    });
}

int s2p_smem(int Wo);

int s2_halo_max(int Wo) { return ((C3_BM - 1 + Wo - 1) / Wo + 2) * Wo; }
int s2_smem(int Wo) { return (s2_halo_max(Wo) + 1) * 128 + 2 * S2_NB * 128; }

int s2p_smem(int Wo) { return (s2_halo_max(Wo) + 1) * 128 + 2 * 64 * 128; }

template <int EPI>
int s2p_launch(C3Args a, hipStream_t st) {
    static int attr_done = 0;
    const int sm = s2p_smem(a.W);
    if (sm > attr_done) {
        (void)hipFuncSetAttribute((const void*)conv3x3s2_dgrad_pair_kernel<EPI>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        attr_done = sm;
    }
    a.ntiles = a.N / 64;
    hipLaunchKernelGGL((conv3x3s2_dgrad_pair_kernel<EPI>), dim3(a.tiles * a.ntiles * 2), dim3(256), sm, st, a);
    PDNN_LAUNCH_RET;
}

template <bool DG, int EPI, bool PRE, bool FP>
int s2_launch(const C3Args& a, hipStream_t st) {
    static int attr_done = 0;
    const int sm = s2_smem(a.W);
    if (sm > attr_done) {
        (void)hipFuncSetAttribute((const void*)conv3x3s2_kernel<DG, EPI, PRE, FP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        attr_done = sm;
    }
    const int grid = a.tiles * a.ntiles * (DG ? 4 : 1);
    hipLaunchKernelGGL((conv3x3s2_kernel<DG, EPI, PRE, FP>), dim3(grid), dim3(256), sm, st, a);
    PDNN_LAUNCH_RET;
}

FastDiv s2_fdiv(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}

}  // namespace

// Whether the stride-2 halo kernels take the conv of an H x W x C input with N output channels, in both directions:
// H, W even (output Ho = H / 2, Wo = W / 2), C and N multiples of 128 (each is the staged reduction of one direction
// and the 128-wide output tile of the other), the halo + weight buffers within 80 KB (two blocks per CU).
PDNN_API int pdnn_conv3x3s2_supported(int Nimg, int H, int W, int C, int N) {
    if (H % 2 || W % 2 || H < 2 || W < 2 || C % S2_NB || C < S2_NB || N % S2_NB || N < S2_NB) return 0;
    if ((long)Nimg * H * W >= (1L << 31) / 2) return 0;
    return s2_smem(W / 2) <= 80 * 1024 ? 1 : 0;
}

// Forward (dgrad = 0): y [Nimg][H/2][W/2][N] = conv3x3/s2/p1(x [Nimg][H][W][C], w [N][3][3][C]); stats: the output's
// BN statistics bins (else plain); pro_sc / pro_sh: x is the pre-activation t of relu(t * sc + sh), applied while
// staging, and written to pre_out [Nimg][H][W][C] when given (the activation the weight gradient reads).
// Data gradient (dgrad = 1): x = dy [Nimg][H/2][W/2][C] (C = the conv's output channels K), w = conv3x3_flip's
// W' [N][3][3][C] (N = the conv's input channels), y = dx [Nimg][H][W][N]; bn_x (with stats): the fused BN backward
// of the layer that produced the conv's input (gm = dx * mask, sums into stats); pre_*: the BN-backward apply of dy's
// own BatchNorm in the operand staging (dt written to pre_out).  pair: the data gradient without the prologue on the
// class-pair kernel (two parity classes per block).
PDNN_API int pdnn_conv3x3s2(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nimg, int H, int W, int C, int N,
                            int dgrad, float* stats, const bf16_t* bn_x, const float* bn_mean, const float* bn_invstd,
                            const float* bn_mscale, const float* bn_mshift, const bf16_t* pre_t,
                            const float* pre_mean, const float* pre_invstd, const float* pre_gamma,
                            const float* pre_dgamma, const float* pre_dbeta, bf16_t* pre_out, const float* pro_sc,
                            const float* pro_sh, int pair, hipStream_t st) {
    if (!pdnn_conv3x3s2_supported(Nimg, H, W, dgrad ? N : C, dgrad ? C : N)) return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y;
    a.Nimg = Nimg; a.H = H / 2; a.W = W / 2; a.C = C; a.N = N; a.P = Nimg * a.H * a.W;
    a.dW = s2_fdiv(a.W); a.dH = s2_fdiv(a.H);
    a.tiles = (int)cdiv(a.P, C3_BM);
    a.ntiles = N / S2_NB;
    a.halo_max = s2_halo_max(a.W);
    a.stats = stats;
    a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
    a.pre_t = pre_t; a.pre_mean = pre_mean; a.pre_invstd = pre_invstd; a.pre_gamma = pre_gamma;
    a.pre_dgamma = pre_dgamma; a.pre_dbeta = pre_dbeta; a.pre_out = pre_out;
    a.pro_sc = pro_sc; a.pro_sh = pro_sh;
    if (!pro_sc != !pro_sh || (bn_x && !stats)) return (int)hipErrorInvalidValue;
    if (pre_t && !(pre_mean && pre_invstd && pre_dgamma && pre_dbeta)) return (int)hipErrorInvalidValue;
    // pre_out: dt of the data gradient's BN-backward prologue, or (forward with pro_sc) the prologue's output a1
    if (pre_out && !pre_t && !(pro_sc && !dgrad)) return (int)hipErrorInvalidValue;
    if (dgrad) {
        if (pro_sc) return (int)hipErrorInvalidValue;
        if (pair && !pre_t) return bn_x ? s2p_launch<C3_BNB>(a, st) : (stats ? (int)hipErrorInvalidValue : s2p_launch<C3_PLAIN>(a, st));
        if (bn_x) return pre_t ? s2_launch<true, C3_BNB, true, false>(a, st) : s2_launch<true, C3_BNB, false, false>(a, st);
        if (stats) return (int)hipErrorInvalidValue;
        return pre_t ? s2_launch<true, C3_PLAIN, true, false>(a, st) : s2_launch<true, C3_PLAIN, false, false>(a, st);
    }
    if (pre_t || bn_x) return (int)hipErrorInvalidValue;
    if (pro_sc) return stats ? s2_launch<false, C3_STATS, false, true>(a, st) : s2_launch<false, C3_PLAIN, false, true>(a, st);
    return stats ? s2_launch<false, C3_STATS, false, false>(a, st) : s2_launch<false, C3_PLAIN, false, false>(a, st);
}
