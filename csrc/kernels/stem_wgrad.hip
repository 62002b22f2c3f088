// Weight gradient of the ImageNet stem (7x7 / stride 2 / pad 3, 3 -> 64 channels) read straight from the
// NCHW bf16 batch (reference layer: the ResNet ImageNet stem conv, pytorch_code/model_ops/resnet.py stem).
//
//   dW32[n][r][k] = sum over output pixels p of dt[p][n] * A_r[p][k],   k = c * 8 + j  (stem.hip's NCHW form:
//   A_r[p][c*8 + j] = x[img][c][2 oy - 3 + r][2 ox - 4 + j], channel 3 and j = 0 zero-weight padding)
//
// The implicit-GEMM engine ran this as an im2col weight gradient over the channel-padded NHWC copy
// (K = 7*7*8, 62% of the MFMA work and loads on padding, per-chunk divisions in the gather): 534 us at the very
// end of the backward with the rest of the GPU idle (profiles/resnet50_bs256_timeline_r3b.txt).  Here a block
// takes a run of 96-pixel tiles; per tile it stages dt [96 px][64 n] and the seven A_r [96 px][32 k] images
// (each lane loads 8 input columns of one channel row for one pixel: 16 bytes, word-shifted at the image
// border, exactly like the forward) into LDS, and reduces over the pixels through transpose reads
// (ds_read_b64_tr_b16) of both: 8 waves, wave w owns n-fragment (w & 3), k-half (w >> 2) for all 7 filter
// rows.  The next tile is fetched into registers under the current tile's MFMAs; 96-pixel tiles keep the LDS at
// 66 KB so two blocks share a CU (one block of 128-pixel tiles: 329 us, load-latency bound).  Per-block partials
// [64][7][32] go to a workspace; a second kernel sums them.
#include "conv_direct.h"

namespace {
using namespace pg;

constexpr int SW_NT = 512;
constexpr int SW_BM = 96;                  // pixels per tile (LDS 66 KB: two blocks per CU)
constexpr int SW_R = 7;
constexpr int SW_AP = 80;                  // bytes per pixel row of an A_r image (64 + 16 skew: 2-way tr reads)
constexpr int SW_PS = 64 * SW_R * 32 + 64; // floats per block partial (padded by 256 B)

struct SWArgs {
    const bf16_t* x;     // [Nimg][3][H][W]
    const bf16_t* dt;    // [P][64]; with PRE: the max-pool gradient ga, dt = bn_bwd_apply(ga, t) (mask mode 2)
    float* ws;           // partials
    int H, W, Ho, Wo, P, tiles, G;
    FastDiv dWo, dHo;
    // PRE: the stem BatchNorm's backward apply fused into the dt staging (dt never materialised)
    const bf16_t* t;     // [P][64] BN input
    const float *mean, *invstd, *gamma, *dgamma, *dbeta, *mscale, *mshift;
};

template <bool PRE>
__global__ void __launch_bounds__(SW_NT, 2) stem_wgrad_kernel(SWArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const dimg = reinterpret_cast<bf16_t*>(smem);                 // [96 px][64 n], mimg_off<64>
    char* const aimg = smem + SW_BM * 64 * 2;                              // [7][96 px][SW_AP bytes]
    float* const coef = reinterpret_cast<float*>(aimg + SW_R * SW_BM * SW_AP);   // PRE: [5][64] k, A, B, ms, mh
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if constexpr (PRE) {
        if (tid < 64) {
            const float invL = (float)(1.0 / (double)a.P);
            const float is = a.invstd[tid], k = (a.gamma ? a.gamma[tid] : 1.f) * is;
            const float dg = a.dgamma[tid] * invL, db = a.dbeta[tid] * invL;
            coef[tid] = k;
            coef[64 + tid] = -k * is * dg;
            coef[128 + tid] = k * (a.mean[tid] * is * dg - db);
            coef[192 + tid] = a.mscale[tid];
            coef[256 + tid] = a.mshift[tid];
        }
        __syncthreads();
    }
    const int t0 = (int)((long)blockIdx.x * a.tiles / a.G), t1 = (int)((long)(blockIdx.x + 1) * a.tiles / a.G);
    const int fm = wave & 3, kh = wave >> 2;

    f32x4_t acc[SW_R];
#pragma unroll
    for (int r = 0; r < SW_R; ++r) acc[r] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // staging roles: dt chunks i = tid, tid + 512 (pixel i >> 3, chunk i & 7; i < 768); A: pixel tid >> 2 (< 96),
    // channel tid & 3, all 7 filter rows
    u16x8_t rd[2], ra[SW_R], rt[PRE ? 2 : 1];
    uint32_t okm = 0;                          // bits 0-1: dt chunk valid (masked at the LDS store)
    const long plane = (long)a.H * a.W;
    auto load_regs = [&](int t) {
        const int p0 = t * SW_BM;
        const int plast = min(a.P, p0 + SW_BM) - 1;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + j * SW_NT, p = p0 + (i >> 3);
            const bool ok = p < a.P && i < SW_BM * 8;
            rd[j] = *reinterpret_cast<const u16x8_t*>(a.dt + (long)(ok ? p : plast) * 64 + (i & 7) * 8);
            if constexpr (PRE) rt[j] = *reinterpret_cast<const u16x8_t*>(a.t + (long)(ok ? p : plast) * 64 + (i & 7) * 8);
            okm = ok ? (okm | (1u << j)) : (okm & ~(1u << j));
        }
        const int p = min(p0 + min(tid >> 2, SW_BM - 1), plast), c = tid & 3;
        const int q = (int)fdiv((uint32_t)p, a.dWo);
        const int ox = p - q * a.Wo;
        const int img = (int)fdiv((uint32_t)q, a.dHo);
        const int oy = q - img * a.Ho;
        const int lo = 2 * ox - 4;
        const int col = lo < 0 ? 0 : (lo + 8 > a.W ? a.W - 8 : lo);
        const int sh = (col - lo) / 2;         // +2 / +1 / -1 words at the borders, 0 inside
        const bf16_t* rowp = a.x + ((long)img * 3 + (c < 3 ? c : 0)) * plane + col;
#pragma unroll
        for (int r = 0; r < SW_R; ++r) {
            const int iy = 2 * oy - 3 + r;
            const bool rok = c < 3 && (unsigned)iy < (unsigned)a.H;
            const uint4 w = __builtin_bit_cast(uint4, *reinterpret_cast<const u16x8_t*>(rowp + (long)(rok ? iy : 0) * a.W));
            const uint32_t m = rok ? 0xFFFFFFFFu : 0u;
            uint4 o;
            o.x = (sh == 0 ? w.x : sh == 1 ? 0u : sh == 2 ? 0u : w.y) & m;
            o.y = (sh == 0 ? w.y : sh == 1 ? w.x : sh == 2 ? 0u : w.z) & m;
            o.z = (sh == 0 ? w.z : sh == 1 ? w.y : sh == 2 ? w.x : w.w) & m;
            o.w = (sh == 0 ? w.w : sh == 1 ? w.z : sh == 2 ? w.y : 0u) & m;
            ra[r] = __builtin_bit_cast(u16x8_t, o);
        }
    };
    auto store_lds = [&]() {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + j * SW_NT;
            if (i < SW_BM * 8) {
                u16x8_t v = rd[j];
                if constexpr (PRE) {     // dt = k * gm + A * t + B, gm = ga * [t * ms + mh > 0] (bn_bwd_apply mode 2)
                    const float* cf = coef + (i & 7) * 8;
                    float gm[8], tv[8], o[8];
                    unpack8(rd[j], gm);
                    unpack8(rt[j], tv);
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float g0 = fmaf(tv[e], cf[192 + e], cf[256 + e]) > 0.f ? gm[e] : 0.f;
                        o[e] = fmaf(cf[e], g0, fmaf(tv[e], cf[64 + e], cf[128 + e]));
                    }
                    v = pack8(o);
                }
                *reinterpret_cast<u16x8_t*>(dimg + mimg_off<64>(i >> 3, i & 7)) = mask16(v, (okm >> j) & 1);
            }
        }
        // the A values are finite for every pixel (clamped to the last one): dt's zero rows cancel them
        if (tid < SW_BM * 4) {
#pragma unroll
            for (int r = 0; r < SW_R; ++r)
                *reinterpret_cast<u16x8_t*>(aimg + (r * SW_BM + (tid >> 2)) * SW_AP + (tid & 3) * 16) = ra[r];
        }
    };

    // transpose-read coordinates: rows (pixels) k = 32 ks + 8 g + q (+4), columns (k index) 16 kh + 4 pq .. +3
    const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
    const int abyte = (16 * kh + 4 * pq) * 2;

    if (t0 < t1) {
        load_regs(t0);
        store_lds();
    }
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
        const bool more = t + 1 < t1;
        if (more) load_regs(t + 1);
#pragma unroll
        for (int ks = 0; ks < SW_BM / 32; ++ks) {
            const bf16x8_t af = frag_mnmajor<64>(dimg, fm * 16, ks, lane);
            const int row = ks * 32 + 8 * g + q;
#pragma unroll
            for (int r = 0; r < SW_R; ++r) {
                const char* b = aimg + (r * SW_BM + row) * SW_AP + abyte;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(b + 4 * SW_AP));
                typedef __attribute__((ext_vector_type(8))) short s16x8;
                const s16x8 xv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, __builtin_bit_cast(bf16x8_t, xv), acc[r], 0, 0, 0);
            }
        }
        __syncthreads();
        if (more) {
            store_lds();
            __syncthreads();
        }
    }
    // lane holds dW32[n = 16 fm + 4 g + j][r][k = 16 kh + (lane & 15)]
    float* ws = a.ws + (long)blockIdx.x * SW_PS;
#pragma unroll
    for (int r = 0; r < SW_R; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) ws[((fm * 16 + 4 * g + j) * SW_R + r) * 32 + 16 * kh + (lane & 15)] = acc[r][j];
}

// out[i] = sum over the G block partials (fresh output, [64][7][32] fp32); 32 partial groups per 8 float4s
__global__ void __launch_bounds__(256) stem_wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                                int G, float* __restrict__ acc) {
    constexpr int PG = 32, OUT = 8, TOTAL = 64 * SW_R * 32 / 4;
    __shared__ float4 red[PG][OUT];
    const int o = threadIdx.x % OUT, pg = threadIdx.x / OUT;
    const int i = blockIdx.x * OUT + o;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < TOTAL) {
        const float* src = ws + 4 * i;
        int b = pg;
        for (; b + 7 * PG < G; b += 8 * PG) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float4*>(src + (long)(b + PG * j) * SW_PS);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
        }
        for (; b < G; b += PG) {
            const float4 v = *reinterpret_cast<const float4*>(src + (long)b * SW_PS);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    red[pg][o] = s;
    __syncthreads();
    if (pg == 0 && i < TOTAL) {
#pragma unroll
        for (int k = 1; k < PG; ++k) { const float4 v = red[k][o]; s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
        if (acc) {
            // accumulate straight into the parameter's gradient, [64][3][7][7] in channels-last memory
            // (n*147 + r*21 + s*3 + c): element (n, r, k = c*8 + j) is tap s = j - 1 of channel c
            const float e4[4] = {s.x, s.y, s.z, s.w};
            const int nr = (4 * i) / 32, n = nr / SW_R, r = nr - n * SW_R;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = (4 * i + q) & 31, c = k >> 3, j = k & 7;
                if (c < 3 && j >= 1) acc[n * 147 + r * 21 + (j - 1) * 3 + c] += e4[q];
            }
        } else {
            *reinterpret_cast<float4*>(out + 4 * i) = s;
        }
    }
}

FastDiv sw_fdiv(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}

// blocks (each a fixed run of tiles; two fit a CU): tuning stem_wgrad_blocks.  At the end of the ResNet backward this
// kernel can start while the side stream still holds CUs; a grid of exactly two blocks per CU then leaves a late
// CU with two runs in sequence
int sw_blocks(long P) {
    const long tiles = (P + SW_BM - 1) / SW_BM;
    const long cap = pg::tune().stem_wgrad_blocks;
    return (int)(tiles < cap ? tiles : cap);
}
}  // namespace

// floats of workspace pdnn_stem_wgrad_nchw needs
PDNN_API int pdnn_stem_wgrad_ws(int Nimg, int Ho, int Wo) { return sw_blocks((long)Nimg * Ho * Wo) * SW_PS; }

// dw32 [64][7][32] fp32 (overwritten; k = c*8 + j as pdnn_stem_conv_nchw's weight) = weight gradient of the
// NCHW stem given dt [Nimg*Ho*Wo][64] bf16 (the gradient w.r.t. its output).  t != null: `dt` is the gradient
// ga of the stem's BN+ReLU output and the BN backward apply (mode 2: ReLU mask recomputed from t) runs in the
// staging, so dt is never written.  acc != null: the result is added into acc (the parameter gradient,
// [64][3][7][7] channels-last fp32) instead of written to dw32.
PDNN_API int pdnn_stem_wgrad_nchw(const bf16_t* x, const bf16_t* dt, float* dw32, int Nimg, int H, int W, int Ho,
                                  int Wo, float* ws, const bf16_t* t, const float* mean, const float* invstd,
                                  const float* gamma, const float* dgamma, const float* dbeta, const float* mscale,
                                  const float* mshift, float* acc, hipStream_t st) {
    if (Ho != (H + 6 - 7) / 2 + 1 || Wo != (W + 6 - 7) / 2 + 1 || W % 2 || W < 8 || !ws || (!dw32 && !acc) ||
        (long)Nimg * Ho * Wo >= (1L << 31))
        return (int)hipErrorInvalidValue;
    const bool pre = t != nullptr;
    if (pre && !(mean && invstd && dgamma && dbeta && mscale && mshift)) return (int)hipErrorInvalidValue;
    SWArgs a{};
    a.x = x; a.dt = dt; a.ws = ws;
    a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.P = Nimg * Ho * Wo;
    a.tiles = (int)cdiv(a.P, SW_BM);
    a.G = sw_blocks(a.P);
    a.dWo = sw_fdiv(Wo); a.dHo = sw_fdiv(Ho);
    a.t = t; a.mean = mean; a.invstd = invstd; a.gamma = gamma; a.dgamma = dgamma; a.dbeta = dbeta;
    a.mscale = mscale; a.mshift = mshift;
    const int sm = SW_BM * 64 * 2 + SW_R * SW_BM * SW_AP + (pre ? 5 * 64 * 4 : 0);
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)stem_wgrad_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, sm + 5 * 64 * 4);
        (void)hipFuncSetAttribute((const void*)stem_wgrad_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, sm + 5 * 64 * 4);
        attr = true;
    }
    if (pre) hipLaunchKernelGGL(stem_wgrad_kernel<true>, dim3(a.G), dim3(SW_NT), sm, st, a);
    else hipLaunchKernelGGL(stem_wgrad_kernel<false>, dim3(a.G), dim3(SW_NT), sm, st, a);
    const int e = (int)hipGetLastError();
    if (e) return e;
    hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3((64 * SW_R * 32 / 4 + 7) / 8), dim3(256), 0, st,
                       (const float*)ws, dw32, a.G, acc);
    PDNN_LAUNCH_RET;
}
