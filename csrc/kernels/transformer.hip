// Transformer kernels for the GPT-2 configuration (BASELINE.json config 4):
// LayerNorm forward/backward, causal attention softmax forward/backward (the attention GEMMs run on
// the MFMA engine of gemm_mfma.hip), token + position embedding forward/backward.
//
// Row kernels use one 64-lane wave per row with 16-byte vector loads (Guideline 13); statistics in fp32.
#include "common.h"

namespace {
constexpr int NT = 256;   // 4 rows (waves) per block

// ---------------------------------------------------------------------------------------------- LayerNorm
// D % 8 == 0, D <= 64 * 8 * 4 = 2048.  y = (x - mean) * rstd * gamma + beta ; saves mean, rstd.
template <int MAXC>
__global__ void __launch_bounds__(NT) layernorm_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ g,
                                                           const float* __restrict__ b, bf16_t* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd,
                                                           int rows, int D, float eps) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int CH = D / 8;
    const bf16_t* xr = x + (long)row * D;
    float v[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
        if (c < CH) {
            unpack8(*reinterpret_cast<const u16x8_t*>(xr + c * 8), v[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) s += v[i][j];
        }
    }
    const float mu = wave_sum(s) / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
        if (c < CH) {
#pragma unroll
            for (int j = 0; j < 8; ++j) { const float d = v[i][j] - mu; q += d * d; }
        }
    }
    const float rs = rsqrtf(wave_sum(q) / D + eps);
    if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
        if (c < CH) {
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mu) * rs * g[c * 8 + j] + b[c * 8 + j];
            *reinterpret_cast<u16x8_t*>(y + (long)row * D + c * 8) = pack8(o);
        }
    }
}

// dx = rstd * (gg - mean(gg) - xhat * mean(gg * xhat)) (+ dres, the residual branch), gg = dy * gamma; per-block partial dgamma/dbeta
// into the STAT_BINS statistics bins (common.h: row pair i adds into bin i % 64) -> pdnn_bn_bwd_finalize.
template <int MAXC>
__global__ void __launch_bounds__(NT) layernorm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                           const float* __restrict__ g, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, const bf16_t* __restrict__ dres,
                                                           bf16_t* __restrict__ dx, float* __restrict__ slab, int rows,
                                                           int D) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int CH = D / 8;
    float pb[MAXC][8], pg[MAXC][8], gam[MAXC][8];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            pb[i][j] = pg[i][j] = 0.f;
            gam[i][j] = c < CH ? g[c * 8 + j] : 0.f;          // gamma of this lane's channels, once
        }
    }
    // a wave walks rows row0, row0 + stride, ...: the next row's dy / x / dres / statistics are loaded before this
    // row's dx is stored (the loads of a row used to start only after the previous row's stores and its own
    // reductions: 17 us for GPT-2's 8192 x 768, ~2 TB/s)
    const int stride = gridDim.x * (NT / 64);
    int row = blockIdx.x * (NT / 64) + w;
    u16x8_t cdy[MAXC], cx[MAXC], cr[MAXC];
    float cmu = 0.f, crs = 0.f;
    auto load = [&](int r, u16x8_t (&dyv)[MAXC], u16x8_t (&xv)[MAXC], u16x8_t (&rv)[MAXC], float& mu, float& rs) {
        const int rr = r < rows ? r : rows - 1;                // clamped: a past-the-end prefetch reads a valid row
        mu = mean[rr];
        rs = rstd[rr];
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = lane + 64 * i;
            if (c < CH) {
                dyv[i] = *reinterpret_cast<const u16x8_t*>(dy + (long)rr * D + c * 8);
                xv[i] = *reinterpret_cast<const u16x8_t*>(x + (long)rr * D + c * 8);
                if (dres) rv[i] = *reinterpret_cast<const u16x8_t*>(dres + (long)rr * D + c * 8);
            }
        }
    };
    if (row < rows) load(row, cdy, cx, cr, cmu, crs);
    for (; row < rows; row += stride) {
        u16x8_t ndy[MAXC], nx[MAXC], nr[MAXC];
        float nmu, nrs;
        load(row + stride, ndy, nx, nr, nmu, nrs);
        const float mu = cmu, rs = crs;
        float gv[MAXC][8], xh[MAXC][8];
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = lane + 64 * i;
            if (c < CH) {
                float xv[8];
                unpack8(cdy[i], gv[i]);
                unpack8(cx[i], xv);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    xh[i][j] = (xv[j] - mu) * rs;
                    pb[i][j] += gv[i][j];
                    pg[i][j] += gv[i][j] * xh[i][j];
                    const float gg = gv[i][j] * gam[i][j];
                    s1 += gg;
                    s2 += gg * xh[i][j];
                }
            }
        }
        s1 = wave_sum(s1) / D;
        s2 = wave_sum(s2) / D;
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            const int c = lane + 64 * i;
            if (c < CH) {
                float o[8], rr[8];
                if (dres) unpack8(cr[i], rr);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    o[j] = rs * (gv[i][j] * gam[i][j] - s1 - xh[i][j] * s2) + (dres ? rr[j] : 0.f);
                *reinterpret_cast<u16x8_t*>(dx + (long)row * D + c * 8) = pack8(o);
            }
        }
#pragma unroll
        for (int i = 0; i < MAXC; ++i) {
            cdy[i] = ndy[i];
            cx[i] = nx[i];
            cr[i] = nr[i];
        }
        cmu = nmu;
        crs = nrs;
    }
    // block-level combine of the 4 waves' column partials, then one slab row pair per block
    __shared__ float red[2][NT / 64][MAXC * 512];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
        if (c < CH)
#pragma unroll
            for (int j = 0; j < 8; ++j) { red[0][w][c * 8 + j] = pb[i][j]; red[1][w][c * 8 + j] = pg[i][j]; }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += NT) {
        float a = 0.f, bb = 0.f;
        for (int k = 0; k < NT / 64; ++k) { a += red[0][k][d]; bb += red[1][k][d]; }
        float* row = stat_row(slab, blockIdx.x, D);          // STAT_BINS bins (common.h), finalized like BN's
        stat_add(row + d, a);
        stat_add(row + D + d, bb);
    }
}

// ---------------------------------------------------------------------------------------------- softmax
// P[r][k] = softmax_k(S[r][k] * scale) over k <= q (causal, q = r % T), 0 elsewhere; lse[r] saved.
// One wave per row, T <= 64 * 32.
__global__ void __launch_bounds__(NT) attn_softmax_fwd_kernel(const float* __restrict__ S, long ldS,
                                                              bf16_t* __restrict__ P, long ldP,
                                                              float* __restrict__ lse, int rows, int T, float scale,
                                                              int causal) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int q = r % T;
    const int lim = causal ? q + 1 : T;
    const float* s = S + (long)r * ldS;
    float m = -INFINITY;
    for (int k = lane * 4; k < T; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(s + k);
        const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k + j < lim) m = fmaxf(m, a[j] * scale);
    }
    m = wave_max(m);
    float sum = 0.f;
    for (int k = lane * 4; k < T; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(s + k);
        const float a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k + j < lim) sum += __expf(a[j] * scale - m);
    }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
    if (lane == 0) lse[r] = m + __logf(sum);
    bf16_t* p = P + (long)r * ldP;
    for (int k = lane * 4; k < T; k += 256) {
        const float4 v = *reinterpret_cast<const float4*>(s + k);
        const float a[4] = {v.x, v.y, v.z, v.w};
        u16x4_t o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = f2bf(k + j < lim ? __expf(a[j] * scale - m) * inv : 0.f);
        *reinterpret_cast<u16x4_t*>(p + k) = o;
    }
}

// dS[r][k] = scale * P[r][k] * (dP[r][k] - delta[r]),  delta[r] = sum_k P[r][k] dP[r][k].
// causal: only k <= q (q = r % T) is read -- the causal dP GEMM skips the tiles above the diagonal, whose memory is
// never written (0 * a NaN bit pattern left there would poison delta); dS is 0 above the diagonal.
__global__ void __launch_bounds__(NT) attn_softmax_bwd_kernel(const bf16_t* __restrict__ P, long ldP,
                                                              const float* __restrict__ dP, long lddP,
                                                              bf16_t* __restrict__ dS, long lddS, int rows, int T,
                                                              float scale, int causal) {
    const int lane = threadIdx.x & 63;
    const int r = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int lim = causal ? r % T + 1 : T;
    const bf16_t* p = P + (long)r * ldP;
    const float* dp = dP + (long)r * lddP;
    float d = 0.f;
    for (int k = lane * 4; k < T; k += 256) {
        if (k >= lim) break;
        const u16x4_t pv = *reinterpret_cast<const u16x4_t*>(p + k);
        const float4 g = *reinterpret_cast<const float4*>(dp + k);
        const float gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k + j < lim) d += bf2f(pv[j]) * gg[j];
    }
    d = wave_sum(d);
    bf16_t* o = dS + (long)r * lddS;
    for (int k = lane * 4; k < T; k += 256) {
        u16x4_t out = {0, 0, 0, 0};
        if (k < lim) {
            const u16x4_t pv = *reinterpret_cast<const u16x4_t*>(p + k);
            const float4 g = *reinterpret_cast<const float4*>(dp + k);
            const float gg[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) out[j] = k + j < lim ? f2bf(scale * bf2f(pv[j]) * (gg[j] - d)) : (bf16_t)0;
        }
        *reinterpret_cast<u16x4_t*>(o + k) = out;
    }
}

// ---------------------------------------------------------------------------------------------- embedding
// out[r] = wte[idx[r]] + wpe[r % T]   (bf16 tables: the optimizer-maintained weight shadows)
__global__ void __launch_bounds__(NT) embedding_fwd_kernel(const int64_t* __restrict__ idx,
                                                           const bf16_t* __restrict__ wte,
                                                           const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out,
                                                           int rows, int T, int D) {
    const int CH = D / 8;
    const long total = (long)rows * CH;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        const long r = i / CH;
        const int c = (int)(i - r * CH) * 8;
        float a[8], b[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(wte + idx[r] * D + c), a);
        if (wpe) {
            unpack8(*reinterpret_cast<const u16x8_t*>(wpe + (long)(r % T) * D + c), b);
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] += b[j];
        }
        *reinterpret_cast<u16x8_t*>(out + r * D + c) = pack8(a);
    }
}

// dwte[idx[r]] += sc * g[r] (fp32 atomics; rows hitting the same token accumulate), dwpe[r % T] += g[r]; either
// table may be absent (the split tied-embedding path reduces dwpe and the wte rows separately: parallel/ddp.py)
__global__ void __launch_bounds__(NT) embedding_bwd_kernel(const int64_t* __restrict__ idx,
                                                           const bf16_t* __restrict__ g, float* __restrict__ dwte,
                                                           float* __restrict__ dwpe, int rows, int T, int D, float sc) {
    const long total = (long)rows * D;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        const long r = i / D;
        const int c = (int)(i - r * D);
        const float v = bf2f(g[i]);
        if (dwte) atomicAdd(dwte + idx[r] * D + c, sc * v);
        if (dwpe) atomicAdd(dwpe + (long)(r % T) * D + c, v);
    }
}
}  // namespace

PDNN_API int pdnn_layernorm_fwd(const bf16_t* x, const float* g, const float* b, bf16_t* y, float* mean, float* rstd,
                                int rows, int D, float eps, hipStream_t st) {
    const dim3 grid((rows + 3) / 4);
    if (D % 8 || D > 2048) return (int)hipErrorInvalidValue;
    if (D <= 512)
        hipLaunchKernelGGL(layernorm_fwd_kernel<1>, grid, dim3(NT), 0, st, x, g, b, y, mean, rstd, rows, D, eps);
    else if (D <= 1024)
        hipLaunchKernelGGL(layernorm_fwd_kernel<2>, grid, dim3(NT), 0, st, x, g, b, y, mean, rstd, rows, D, eps);
    else
        hipLaunchKernelGGL(layernorm_fwd_kernel<4>, grid, dim3(NT), 0, st, x, g, b, y, mean, rstd, rows, D, eps);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_layernorm_bwd_blocks(int rows) { return rows / 16 < 1 ? 1 : (rows / 16 > 512 ? 512 : rows / 16); }

PDNN_API int pdnn_layernorm_bwd(const bf16_t* dy, const bf16_t* x, const float* g, const float* mean,
                                const float* rstd, const bf16_t* dres, bf16_t* dx, float* slab, int rows, int D,
                                int nblocks, hipStream_t st) {
    if (D % 8 || D > 2048) return (int)hipErrorInvalidValue;
    const dim3 grid(nblocks);
    if (D <= 512)
        hipLaunchKernelGGL(layernorm_bwd_kernel<1>, grid, dim3(NT), 0, st, dy, x, g, mean, rstd, dres, dx, slab, rows, D);
    else if (D <= 1024)
        hipLaunchKernelGGL(layernorm_bwd_kernel<2>, grid, dim3(NT), 0, st, dy, x, g, mean, rstd, dres, dx, slab, rows, D);
    else
        hipLaunchKernelGGL(layernorm_bwd_kernel<4>, grid, dim3(NT), 0, st, dy, x, g, mean, rstd, dres, dx, slab, rows, D);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_attn_softmax_fwd(const float* S, long ldS, bf16_t* P, long ldP, float* lse, int rows, int T,
                                   float scale, int causal, hipStream_t st) {
    if (T % 4 || ldS % 4 || ldP % 4) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(attn_softmax_fwd_kernel, dim3((rows + 3) / 4), dim3(NT), 0, st, S, ldS, P, ldP, lse, rows, T,
                       scale, causal);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_attn_softmax_bwd(const bf16_t* P, long ldP, const float* dP, long lddP, bf16_t* dS, long lddS,
                                   int rows, int T, float scale, int causal, hipStream_t st) {
    if (T % 4) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((rows + 3) / 4), dim3(NT), 0, st, P, ldP, dP, lddP, dS, lddS,
                       rows, T, scale, causal);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_embedding_fwd(const int64_t* idx, const bf16_t* wte, const bf16_t* wpe, bf16_t* out, int rows,
                                int T, int D, hipStream_t st) {
    hipLaunchKernelGGL(embedding_fwd_kernel, dim3(stream_grid((long)rows * (D / 8), NT)), dim3(NT), 0, st, idx, wte,
                       wpe, out, rows, T, D);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_embedding_bwd(const int64_t* idx, const bf16_t* g, float* dwte, float* dwpe, int rows, int T, int D,
                                hipStream_t st) {
    hipLaunchKernelGGL(embedding_bwd_kernel, dim3(stream_grid((long)rows * D, NT)), dim3(NT), 0, st, idx, g, dwte,
                       dwpe, rows, T, D, 1.f);
    PDNN_LAUNCH_RET;
}

// the same with the wte rows scaled by sc (dwte or dwpe may be null)
PDNN_API int pdnn_embedding_bwd_scaled(const int64_t* idx, const bf16_t* g, float* dwte, float* dwpe, int rows, int T,
                                       int D, float sc, hipStream_t st) {
    if (D < 1 || T < 1 || rows < 0) return (int)hipErrorInvalidValue;
    if (rows == 0) return 0;
    hipLaunchKernelGGL(embedding_bwd_kernel, dim3(stream_grid((long)rows * D, NT)), dim3(NT), 0, st, idx, g, dwte,
                       dwpe, rows, T, D, sc);
    PDNN_LAUNCH_RET;
}
