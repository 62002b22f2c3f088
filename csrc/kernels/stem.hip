// ResNet ImageNet stem on gfx950: the 7x7 / stride-2 / pad-3 convolution of the (channel-padded) image and
// the BN-apply + ReLU + 3x3 / stride-2 max-pool that follows it.
//
// conv: the implicit-GEMM engine ran this layer as a generic gather GEMM at 460 us per step (K = 7*7*8
// taps gathered 16 bytes at a time through L1, r3_17 PMC: 0.4 PFLOP/s on 3.2 M output pixels).  Here the
// reduction is ordered filter row by filter row: for one output pixel and filter row r the 7 taps x 8
// channels are 7 CONSECUTIVE input pixels of one NHWC row (112 contiguous bytes), padded to 8 pixels
// (a 64-deep k-chunk, the 8th tap has zero weight).  Each lane's MFMA operand piece (8 k = one input
// pixel's 8 channels, 16 bytes) is loaded straight from global memory in fragment order -- no LDS for
// the activations, neighbouring output pixels' loads overlap in L1/L2 -- and the next filter row's pieces
// are in flight under the current row's MFMAs.  The weights ([7 rows][64 n][64 k], 56 KB) stay resident
// in LDS for a persistent block that walks a contiguous range of pixel tiles of its XCD (adjacent tiles
// share input rows in that XCD's L2).  Epilogue: bf16 store + BN partial statistics (conv_direct.h).
//
// pool: y = maxpool3x3s2(relu(t * scale + shift)) with the window argmax, reading t once; the backward
// recomputes the ReLU mask from t (BatchNorm-backward mask mode 2), so neither the activation nor its
// mask bits are materialised.  Bitwise equal to bn_apply + maxpool_fwd.
// Reference: pytorch_code/model_ops/resnet.py:93-99 (conv1 / bn1 of the ImageNet-layout ResNets).
#include "conv_direct.h"

namespace {
using namespace pg;

constexpr int STEM_C = 8, STEM_N = 64, STEM_R = 7;

struct StemGeo {
    int H, W, Ho, Wo;
    FastDiv dWo, dHo;
};

template <int EPI>
__global__ void __launch_bounds__(256, 2) stem7_kernel(C3Args a, StemGeo g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const wimg = reinterpret_cast<bf16_t*>(smem);         // [7 r][64 n][64 k] kimg_off images
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // weights [64][7][7][8] -> per filter row r a K-major image, k = s*8 + c (s = 7: zero)
    for (int i = tid; i < STEM_R * 64 * 8; i += 256) {
        const int r = i >> 9, n = (i >> 3) & 63, q = i & 7;
        u16x8_t v = c3_zero8();
        if (q < 7) v = *reinterpret_cast<const u16x8_t*>(a.w + ((n * STEM_R + r) * STEM_R + q) * STEM_C);
        *reinterpret_cast<u16x8_t*>(wimg + r * 4096 + kimg_off(n, q)) = v;
    }
    __syncthreads();

    // XCD-contiguous tile ranges: the blocks of XCD x (blockIdx % 8 under round-robin dispatch) walk tiles
    // [x*T8, (x+1)*T8) together, so concurrently running tiles are neighbours
    const int x8 = blockIdx.x & 7, l = blockIdx.x >> 3, G = gridDim.x >> 3;
    const int T8 = (a.tiles + 7) / 8;
    const int t_end = min(a.tiles, (x8 + 1) * T8);
    const int s_lane = lane >> 4;                          // + 4*ks2: this lane's tap s within the filter row

    for (int tile = x8 * T8 + l; tile < t_end; tile += G) {
        const int p0 = tile * C3_BM;
        long ibase[4];
        int oy2[4], ox2[4];
        bool pv[4];
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const int p = p0 + wave * 64 + fm * 16 + (lane & 15);
            pv[fm] = p < a.P;
            const int pp = pv[fm] ? p : a.P - 1;
            const int q = (int)fdiv((uint32_t)pp, g.dWo);
            const int ox = pp - q * g.Wo;
            const int n = (int)fdiv((uint32_t)q, g.dHo);
            const int oy = q - n * g.Ho;
            ibase[fm] = (long)n * g.H * g.W * STEM_C;
            oy2[fm] = 2 * oy - 3;
            ox2[fm] = 2 * ox - 3;
        }
        auto load_row = [&](int r, u16x8_t (&dst)[2][4]) {
#pragma unroll
            for (int ks2 = 0; ks2 < 2; ++ks2)
#pragma unroll
                for (int fm = 0; fm < 4; ++fm) {
                    const int iy = oy2[fm] + r, ix = ox2[fm] + ks2 * 4 + s_lane;
                    const bool ok = pv[fm] && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W;
                    const long off = ok ? ibase[fm] + ((long)iy * g.W + ix) * STEM_C : 0;
                    dst[ks2][fm] = mask16(*reinterpret_cast<const u16x8_t*>(a.x + off), ok);
                }
        };
        f32x4_t acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        u16x8_t cur[2][4], nxt[2][4];
        load_row(0, cur);
#pragma unroll 1
        for (int r = 0; r < STEM_R; ++r) {         // rolled: unrolled, every row's loads were hoisted (spills)
            if (r + 1 < STEM_R) load_row(r + 1, nxt);     // next filter row under this row's MFMAs
            const bf16_t* B = wimg + r * 4096;
#pragma unroll
            for (int ks2 = 0; ks2 < 2; ++ks2) {
                bf16x8_t bfr[4];
#pragma unroll
                for (int f = 0; f < 4; ++f) bfr[f] = frag_kmajor(B, f * 16 + (lane & 15), ks2, lane);
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                    for (int fn = 0; fn < 4; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            bfr[fn], __builtin_bit_cast(bf16x8_t, cur[ks2][fm]), acc[fm][fn], 0, 0, 0);
            }
            if (r + 1 < STEM_R) {
#pragma unroll
                for (int ks2 = 0; ks2 < 2; ++ks2)
#pragma unroll
                    for (int fm = 0; fm < 4; ++fm) cur[ks2][fm] = nxt[ks2][fm];
            }
        }
        c3_epilogue<64, EPI>(a, acc, tile, p0, 0, wave, lane, pv);
    }
}

// The same conv reading the data loader's NCHW bf16 batch directly (3 channels, W even): per filter row r
// the reduction runs over k = c*8 + j (c < 4, the 4th channel zero; j = 0..7 <-> input column 2*ox - 4 + j,
// tap s = j - 1, j = 0 has zero weight), 32 deep = ONE MFMA k-step per filter row.  A lane's operand piece
// is 8 consecutive input columns of one channel row -- 16 bytes, 4-byte aligned because 2*ox - 4 is even --
// so the layer runs 7 k-steps instead of the NHWC form's 14 (channel padding 3 -> 8) and the NCHW -> NHWC
// conversion pass leaves the critical path.  Lanes whose 8 columns cross the left / right image border
// (3 output columns per row) load the nearest in-image 16 bytes, word-shifted.  All 7 rows in flight.
// weight image of the NCHW stem: [7 r][64 n][32 k] bf16, 16-byte chunk q (4 per row) at q ^ ((n >> 1) & 3)
__device__ __forceinline__ int w32_off(int n, int q) { return n * 32 + ((q ^ ((n >> 1) & 3)) << 3); }

template <int EPI>
__global__ void __launch_bounds__(256, 2) stem7n_kernel(C3Args a, StemGeo g) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const wimg = reinterpret_cast<bf16_t*>(smem);         // [7 r][64 n][32 k]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // weights [64][7][32] (k = c*8 + j, built by the host wrapper) -> per-row K-major images
    for (int i = tid; i < STEM_R * 64 * 4; i += 256) {
        const int r = i >> 8, n = (i >> 2) & 63, q = i & 3;
        *reinterpret_cast<u16x8_t*>(wimg + r * 2048 + w32_off(n, q)) =
            *reinterpret_cast<const u16x8_t*>(a.w + (n * STEM_R + r) * 32 + q * 8);
    }
    __syncthreads();
    const int x8 = blockIdx.x & 7, l = blockIdx.x >> 3, G = gridDim.x >> 3;
    const int T8 = (a.tiles + 7) / 8;
    const int t_end = min(a.tiles, (x8 + 1) * T8);
    const int c = lane >> 4;                               // this lane's input channel (3: zero)
    const long plane = (long)g.H * g.W;

    for (int tile = x8 * T8 + l; tile < t_end; tile += G) {
        const int p0 = tile * C3_BM;
        bool pv[4];
        const bf16_t* rowp[4];                            // filter row 0 of this lane's pixel, column `col`
        int iy0[4], shw[4];
        bool cok[4];
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const int p = p0 + wave * 64 + fm * 16 + (lane & 15);
            pv[fm] = p < a.P;
            const int pp = pv[fm] ? p : a.P - 1;
            const int q = (int)fdiv((uint32_t)pp, g.dWo);
            const int ox = pp - q * g.Wo;
            const int nimg = (int)fdiv((uint32_t)q, g.dHo);
            const int oy = q - nimg * g.Ho;
            const int lo = 2 * ox - 4;                     // column of j = 0
            cok[fm] = pv[fm] && c < 3;
            // border lanes (ox = 0, 1 and the last column) load the nearest in-image 16 bytes and shift them
            // by whole 32-bit words (zeros shifted in): shw = +2 / +1 / -1 words, 0 inside
            const int col = lo < 0 ? 0 : (lo + 8 > g.W ? g.W - 8 : lo);
            shw[fm] = (col - lo) / 2;
            iy0[fm] = 2 * oy - 3;
            rowp[fm] = a.x + ((long)nimg * 3 + (c < 3 ? c : 0)) * plane + col;
        }
        auto load_row = [&](int r, u16x8_t (&dst)[4]) {
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
                const int iy = iy0[fm] + r;
                const bool rok = cok[fm] && (unsigned)iy < (unsigned)g.H;
                const uint4 w = __builtin_bit_cast(uint4, *reinterpret_cast<const u16x8_t*>(rowp[fm] + (long)(rok ? iy : 0) * g.W));
                const uint32_t m = rok ? 0xFFFFFFFFu : 0u;
                const int sh = shw[fm];
                uint4 o;
                o.x = (sh == 0 ? w.x : sh == 1 ? 0u : sh == 2 ? 0u : w.y) & m;
                o.y = (sh == 0 ? w.y : sh == 1 ? w.x : sh == 2 ? 0u : w.z) & m;
                o.z = (sh == 0 ? w.z : sh == 1 ? w.y : sh == 2 ? w.x : w.w) & m;
                o.w = (sh == 0 ? w.w : sh == 1 ? w.z : sh == 2 ? w.y : 0u) & m;
                dst[fm] = __builtin_bit_cast(u16x8_t, o);
            }
        };
        f32x4_t acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        // every filter row's pieces in flight at once (28 loads per lane): one memory latency per tile
        u16x8_t v[STEM_R][4];
#pragma unroll
        for (int r = 0; r < STEM_R; ++r) load_row(r, v[r]);
#pragma unroll
        for (int r = 0; r < STEM_R; ++r) {
            bf16x8_t bfr[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const int n = f * 16 + (lane & 15);
                bfr[f] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(wimg + r * 2048 + w32_off(n, lane >> 4)));
            }
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < 4; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], __builtin_bit_cast(bf16x8_t, v[r][fm]),
                                                                          acc[fm][fn], 0, 0, 0);
        }
        c3_epilogue<64, EPI>(a, acc, tile, p0, 0, wave, lane, pv);
    }
}

// y[n][ho][wo][c] = max over the 3x3 / stride-2 / pad-1 window of bf16(relu(t * scale + shift)), idx = the
// first maximal window position (as maxpool_fwd_kernel); one thread per (output pixel, 8 channels).
__global__ void __launch_bounds__(256) bn_relu_maxpool_kernel(const bf16_t* __restrict__ t,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                              uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                              int Ho, int Wo) {
    const int CG = C >> 3;
    const long total = (long)N * Ho * Wo * CG;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        long q = i;
        const int cg = (int)(q % CG); q /= CG;
        const int wo = (int)(q % Wo); q /= Wo;
        const int ho = (int)(q % Ho);
        const int n = (int)(q / Ho);
        float sc[8], sh[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { sc[j] = scale[cg * 8 + j]; sh[j] = shift[cg * 8 + j]; }
        const bf16_t* tb = t + (long)n * H * W * C + cg * 8;
        u16x8_t raw[3][3];
        bool ok[3][3];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int hi = ho * 2 - 1 + r, wi = wo * 2 - 1 + c;
                ok[r][c] = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
                const long off = ok[r][c] ? ((long)hi * W + wi) * C : 0;
                raw[r][c] = *reinterpret_cast<const u16x8_t*>(tb + off);
            }
        float best[8];
        uint8_t bi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                if (!ok[r][c]) continue;
                float v[8];
                unpack8(raw[r][c], v);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float a = bf2f(f2bf(fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f)));
                    if (a > best[j] || (a != a)) { best[j] = a; bi[j] = (uint8_t)(r * 3 + c); }
                }
            }
        const long o = i * 8;
        *reinterpret_cast<u16x8_t*>(y + o) = pack8(best);
        uint2 packed;
        packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
        packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
        *reinterpret_cast<uint2*>(idx + o) = packed;
    }
}

FastDiv make_fdiv_stem(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}
}  // namespace

// Slab rows (sum / sum-of-squares row pairs) of pdnn_stem_conv's statistics for P output pixels.
PDNN_API int pdnn_stem_stats_rows(long P) { return (int)cdiv(P, C3_BM) * 4; }

// y[P][64] = conv7x7/s2/p3(x) for x [Nimg][H][W][8] bf16 (channels zero-padded), w [64][7][7][8] bf16;
// stats: BN partial sums (pdnn_stem_stats_rows pairs) or null (plain epilogue: eval mode).
PDNN_API int pdnn_stem_conv(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nimg, int H, int W, int Ho, int Wo,
                            float* stats, hipStream_t st) {
    if (Ho != (H + 6 - 7) / 2 + 1 || Wo != (W + 6 - 7) / 2 + 1 || (long)Nimg * Ho * Wo >= (1L << 31) ||
        (long)Nimg * H * W * STEM_C >= (1L << 31) * 8L)
        return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y; a.C = STEM_C; a.N = STEM_N;
    a.P = Nimg * Ho * Wo;
    a.tiles = (int)cdiv(a.P, C3_BM);
    a.ntiles = 1;
    a.stats = stats;
    StemGeo g{H, W, Ho, Wo, make_fdiv_stem(Wo), make_fdiv_stem(Ho)};
    const int sm = STEM_R * 64 * 64 * 2;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)stem7_kernel<C3_STATS>, hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        (void)hipFuncSetAttribute((const void*)stem7_kernel<C3_PLAIN>, hipFuncAttributeMaxDynamicSharedMemorySize, sm);
        attr = true;
    }
    const int cap = 2 * grid_cus();                    // two persistent blocks per CU
    int grid = a.tiles < cap ? a.tiles : cap;
    grid = (grid + 7) / 8 * 8;
    if (stats) hipLaunchKernelGGL(stem7_kernel<C3_STATS>, dim3(grid), dim3(256), sm, st, a, g);
    else hipLaunchKernelGGL(stem7_kernel<C3_PLAIN>, dim3(grid), dim3(256), sm, st, a, g);
    PDNN_LAUNCH_RET;
}

// The NCHW form: x [Nimg][3][H][W] bf16 (W even), w [64][7][32] bf16 (k = c*8 + j, see stem7n_kernel).
PDNN_API int pdnn_stem_conv_nchw(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nimg, int H, int W, int Ho,
                                 int Wo, float* stats, hipStream_t st) {
    if (Ho != (H + 6 - 7) / 2 + 1 || Wo != (W + 6 - 7) / 2 + 1 || W % 2 || W < 8 ||
        (long)Nimg * Ho * Wo >= (1L << 31))
        return (int)hipErrorInvalidValue;
    C3Args a{};
    a.x = x; a.w = w; a.y = y; a.C = 3; a.N = STEM_N;
    a.P = Nimg * Ho * Wo;
    a.tiles = (int)cdiv(a.P, C3_BM);
    a.ntiles = 1;
    a.stats = stats;
    StemGeo g{H, W, Ho, Wo, make_fdiv_stem(Wo), make_fdiv_stem(Ho)};
    const int sm = STEM_R * 64 * 32 * 2;              // 28 KB
    const int cap = 2 * grid_cus();                    // two persistent blocks per CU
    int grid = a.tiles < cap ? a.tiles : cap;
    grid = (grid + 7) / 8 * 8;
    if (stats) hipLaunchKernelGGL(stem7n_kernel<C3_STATS>, dim3(grid), dim3(256), sm, st, a, g);
    else hipLaunchKernelGGL(stem7n_kernel<C3_PLAIN>, dim3(grid), dim3(256), sm, st, a, g);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_bn_relu_maxpool(const bf16_t* t, const float* scale, const float* shift, bf16_t* y, uint8_t* idx,
                                  int N, int H, int W, int C, int Ho, int Wo, hipStream_t st) {
    if (C % 8 || Ho != (H + 2 - 3) / 2 + 1 || Wo != (W + 2 - 3) / 2 + 1) return (int)hipErrorInvalidValue;
    const long work = (long)N * Ho * Wo * (C / 8);
    // one item per thread (no grid-stride loop: a thread's next item's 9 loads would wait for its 2 stores)
    hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3((unsigned)cdiv(work, 256)), dim3(256), 0, st, t, scale, shift, y,
                       idx, N, H, W, C, Ho, Wo);
    PDNN_LAUNCH_RET;
}
