// Pooling kernels, NHWC bf16 (SURVEY.md §2.8 K-08 MaxPool, K-09 AvgPool;
// reference call sites pytorch_code/model_ops/lenet.py:22-25, resnet.py:94).
//
// Max pool saves the winning window position as one byte per output element so the backward is a
// gather (each input position visits the <= ceil(k/s)^2 windows that cover it) — no atomics, and
// deterministic even with overlapping 3x3/s2 windows.
#include "common.h"

namespace {
constexpr int NT = 256;

// 32-bit index math (the grid-stride loop bounds are checked on the host: total < 2^31) and the window
// size as a template parameter (KS=3 for every ResNet stem; KS=0 = runtime k): all KS*KS loads of an
// output issue before the compares, and no 64-bit divisions in the index decomposition (they were
// ~40% of the fwd kernel's instructions).
template <int KS>
__global__ void __launch_bounds__(NT) maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                         int Ho, int Wo, int kr, int st, int pad) {
    const int k = KS ? KS : kr;
    const int CG = C >> 3;
    const int total = N * Ho * Wo * CG;
    for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
        int t = i;
        const int cg = t % CG; t /= CG;
        const int wo = t % Wo; t /= Wo;
        const int ho = t % Ho;
        const int n = t / Ho;
        float best[8];
        uint8_t bi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
        const bf16_t* xb = x + (long)n * H * W * C + cg * 8;
        if constexpr (KS > 0) {
            u16x8_t raw[KS][KS];                     // every in-bounds load of the window in flight at once
            bool ok[KS][KS];
#pragma unroll
            for (int r = 0; r < KS; ++r)
#pragma unroll
                for (int c = 0; c < KS; ++c) {
                    const int hi = ho * st - pad + r, wi = wo * st - pad + c;
                    ok[r][c] = (unsigned)hi < (unsigned)H && (unsigned)wi < (unsigned)W;
                    if (ok[r][c]) raw[r][c] = *reinterpret_cast<const u16x8_t*>(xb + ((long)hi * W + wi) * C);
                }
#pragma unroll
            for (int r = 0; r < KS; ++r)
#pragma unroll
                for (int c = 0; c < KS; ++c) {
                    if (!ok[r][c]) continue;
                    float v[8];
                    unpack8(raw[r][c], v);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (v[j] > best[j] || (v[j] != v[j])) { best[j] = v[j]; bi[j] = (uint8_t)(r * KS + c); }
                }
        } else {
            for (int r = 0; r < k; ++r) {
                const int hi = ho * st - pad + r;
                if ((unsigned)hi >= (unsigned)H) continue;
                for (int c = 0; c < k; ++c) {
                    const int wi = wo * st - pad + c;
                    if ((unsigned)wi >= (unsigned)W) continue;
                    float v[8];
                    unpack8(*reinterpret_cast<const u16x8_t*>(xb + ((long)hi * W + wi) * C), v);
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (v[j] > best[j] || (v[j] != v[j])) { best[j] = v[j]; bi[j] = (uint8_t)(r * k + c); }
                }
            }
        }
        const long o = (long)i * 8;                  // == ((n*Ho + ho)*Wo + wo)*C + cg*8
        *reinterpret_cast<u16x8_t*>(y + o) = pack8(best);
        if (idx) {
            uint2 packed;
            packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
            packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
            *reinterpret_cast<uint2*>(idx + o) = packed;
        }
    }
}

// KS=3, ST=2 (ResNet stem): every input pixel receives from at most 2x2 outputs; those candidates' loads
// are issued together (fixed trip counts), then matched against the stored window index.
template <int KS, int ST>
__global__ void __launch_bounds__(NT) maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                         const uint8_t* __restrict__ idx,
                                                         bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                         int Ho, int Wo, int kr, int str, int pad) {
    const int k = KS ? KS : kr, st = ST ? ST : str;
    const int CG = C >> 3;
    const int total = N * H * W * CG;
    for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
        int t = i;
        const int cg = t % CG; t /= CG;
        const int w = t % W; t /= W;
        const int h = t % H;
        const int n = t / H;
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        // outputs ho with ho*st - pad <= h <= ho*st - pad + k - 1
        const int ho_lo = max(0, (h + pad - k + st) / st), ho_hi = min(Ho - 1, (h + pad) / st);
        const int wo_lo = max(0, (w + pad - k + st) / st), wo_hi = min(Wo - 1, (w + pad) / st);
        if constexpr (KS > 0 && ST > 0) {
            constexpr int NC = (KS + ST - 1) / ST;           // candidate outputs per dimension
            uint2 pk[NC][NC];
            u16x8_t gv[NC][NC];
            bool ok[NC][NC];
#pragma unroll
            for (int a = 0; a < NC; ++a)
#pragma unroll
                for (int b = 0; b < NC; ++b) {
                    const int ho = ho_lo + a, wo = wo_lo + b;
                    ok[a][b] = ho <= ho_hi && wo <= wo_hi;
                    if (ok[a][b]) {
                        const long o = ((long)(n * Ho + ho) * Wo + wo) * C + cg * 8;
                        pk[a][b] = *reinterpret_cast<const uint2*>(idx + o);
                        gv[a][b] = *reinterpret_cast<const u16x8_t*>(dy + o);
                    }
                }
#pragma unroll
            for (int a = 0; a < NC; ++a)
#pragma unroll
                for (int b = 0; b < NC; ++b) {
                    if (!ok[a][b]) continue;
                    const int r = h + pad - (ho_lo + a) * ST, s = w + pad - (wo_lo + b) * ST;
                    const uint8_t want = (uint8_t)(r * KS + s);
                    float g[8];
                    unpack8(gv[a][b], g);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const uint32_t word = j < 4 ? pk[a][b].x : pk[a][b].y;
                        if (((word >> (8 * (j & 3))) & 0xff) == want) acc[j] += g[j];
                    }
                }
            *reinterpret_cast<u16x8_t*>(dx + (long)i * 8) = pack8(acc);
            continue;
        }
        for (int ho = ho_lo; ho <= ho_hi; ++ho) {
            const int r = h + pad - ho * st;
            if (r < 0 || r >= k) continue;
            for (int wo = wo_lo; wo <= wo_hi; ++wo) {
                const int s = w + pad - wo * st;
                if (s < 0 || s >= k) continue;
                const long o = ((long)(n * Ho + ho) * Wo + wo) * C + cg * 8;
                const uint2 p = *reinterpret_cast<const uint2*>(idx + o);
                float g[8];
                unpack8(*reinterpret_cast<const u16x8_t*>(dy + o), g);
                const uint8_t want = (uint8_t)(r * k + s);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t word = j < 4 ? p.x : p.y;
                    if (((word >> (8 * (j & 3))) & 0xff) == want) acc[j] += g[j];
                }
            }
        }
        *reinterpret_cast<u16x8_t*>(dx + (long)i * 8) = pack8(acc);
    }
}

// ResNet stem backward, max-pool gather + the BatchNorm-backward statistics in one pass (3x3 / s2 / p1
// window, even H = 2*Ho, W = 2*Wo).  A thread owns the 2x2 input patch (2ho..2ho+1, 2wo..2wo+1) of one
// 8-channel group: those four pixels receive only from outputs (ho..ho+1, wo..wo+1) — 4 dy / idx loads per
// 4 pixels instead of ~9 — so the patch's 4 dy, 4 idx and 4 pre-BN t loads all issue together.  It writes
// ga = the pooled gradient (bf16) and accumulates the BN-backward sums of mask mode 2 (gm = ga where
// t*mscale + mshift > 0): sum(gm), sum(gm * (t - mean) * invstd), per-block partial rows in the slab layout
// of bn_bwd_reduce ([rows][2][C]).  Replaces maxpool_bwd (write ga) + bn_bwd_reduce<2> (read ga and t
// again) on the serial tail of the ResNet backward.
__global__ void __launch_bounds__(NT) maxpool_bwd_bnred_kernel(
    const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
    const bf16_t* __restrict__ tin, const float* __restrict__ mean, const float* __restrict__ invstd,
    const float* __restrict__ mscale, const float* __restrict__ mshift, float* __restrict__ slab, int N, int Ho,
    int Wo, int C) {
    __shared__ float red[2][NT * 8];
    const int CG = C >> 3, W = 2 * Wo;
    const int total = N * Ho * Wo * CG;
    const int t0 = blockIdx.x * NT + threadIdx.x;
    const int cg = t0 % CG;                              // fixed per thread: the grid stride is a multiple of CG
    float mu[8], is[8], ms[8], mh[8], s[8], q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int c = cg * 8 + j;
        mu[j] = mean[c]; is[j] = invstd[c]; ms[j] = mscale[c]; mh[j] = mshift[c];
        s[j] = 0.f; q[j] = 0.f;
    }
    // software-pipelined: item i + stride's 12 loads are issued before item i's 4 stores (s_waitcnt vmcnt counts
    // stores too and retires in order: loads issued after the stores waited for them every iteration)
    struct Item {
        uint2 pk[2][2];
        u16x8_t gv[2][2], tv[2][2];
    };
    auto load = [&](int i, Item& it) {
        int r = i / CG;
        const int wo = r % Wo; r /= Wo;
        const int ho = r % Ho;
        const int n = r / Ho;
        const bool wn = wo + 1 < Wo, hn = ho + 1 < Ho;
#pragma unroll
        for (int da = 0; da < 2; ++da)
#pragma unroll
            for (int db = 0; db < 2; ++db) {
                const bool ok = (da == 0 || hn) && (db == 0 || wn);
                // rows / columns past the edge read the item's own output (valid address), then are ignored
                const long o = ((long)(n * Ho + ho + (ok ? da : 0)) * Wo + wo + (ok ? db : 0)) * C + cg * 8;
                it.pk[da][db] = *reinterpret_cast<const uint2*>(idx + o);
                it.gv[da][db] = *reinterpret_cast<const u16x8_t*>(dy + o);
                if (!ok) it.pk[da][db] = make_uint2(0xffffffffu, 0xffffffffu);    // no window index matches 0xff
                it.tv[da][db] = *reinterpret_cast<const u16x8_t*>(
                    tin + ((long)(n * 2 * Ho + 2 * ho + da) * W + 2 * wo + db) * C + cg * 8);
            }
    };
    const int stride = gridDim.x * NT;
    Item cur, nxt;
    if (t0 < total) load(t0, cur);
    for (int i = t0; i < total; i += stride) {
        load(i + stride < total ? i + stride : i, nxt);
        int r = i / CG;
        const int wo = r % Wo; r /= Wo;
        const int ho = r % Ho;
        const int n = r / Ho;
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                // pixel (2ho+a, 2wo+b) receives from output (ho+da, wo+db) at window row a+1-2da (col b+1-2db):
                // da = 0 always (row a+1), da = 1 only for a = 1 (row 0)
                float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int da = 0; da <= a; ++da)
#pragma unroll
                    for (int db = 0; db <= b; ++db) {
                        const uint32_t want = (uint32_t)((a + 1 - 2 * da) * 3 + (b + 1 - 2 * db));
                        float g[8];
                        unpack8(cur.gv[da][db], g);
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            const uint32_t word = j < 4 ? cur.pk[da][db].x : cur.pk[da][db].y;
                            if (((word >> (8 * (j & 3))) & 0xffu) == want) acc[j] += g[j];
                        }
                    }
                const u16x8_t packed = pack8(acc);
                *reinterpret_cast<u16x8_t*>(dx + ((long)(n * 2 * Ho + 2 * ho + a) * W + 2 * wo + b) * C + cg * 8) =
                    packed;
                float g[8], tv8[8];
                unpack8(packed, g);                          // the stored (bf16) gradient, as a separate pass reads it
                unpack8(cur.tv[a][b], tv8);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float gm = fmaf(tv8[j], ms[j], mh[j]) > 0.f ? g[j] : 0.f;
                    s[j] += gm;
                    q[j] += gm * (tv8[j] - mu[j]) * is[j];
                }
            }
        cur = nxt;
    }
    const int t = threadIdx.x, RPI = NT / CG;
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][t * 8 + j] = s[j]; red[1][t * 8 + j] = q[j]; }
    __syncthreads();
    for (int cc = t; cc < C; cc += NT) {
        const int gg = cc >> 3, j = cc & 7;
        float a = 0.f, b = 0.f;
        for (int k = 0; k < RPI; ++k) { a += red[0][(k * CG + gg) * 8 + j]; b += red[1][(k * CG + gg) * 8 + j]; }
        float* row = stat_row(slab, blockIdx.x, C);
        stat_add(row + cc, a);
        stat_add(row + C + cc, b);
    }
}

// Global average pool [N][HW][C] -> [N][C] (fp32 accumulate).  One block per (n, 2048-channel slab).
__global__ void __launch_bounds__(NT) avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         int HW, int C) {
    const int n = blockIdx.x;
    const int CG = C >> 3;
    const int RPI = NT / CG > 0 ? NT / CG : 1;
    __shared__ float red[NT * 8];
    const int t = threadIdx.x, cg = t % CG, rr = t / CG;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (CG <= NT && rr < RPI) {
        for (int p = rr; p < HW; p += RPI) {
            float v[8];
            unpack8(*reinterpret_cast<const u16x8_t*>(x + ((long)n * HW + p) * C + cg * 8), v);
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += v[j];
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[t * 8 + j] = s[j];
    __syncthreads();
    const float inv = 1.f / HW;
    for (int c = t; c < C; c += NT) {
        const int g = c >> 3, j = c & 7;
        float a = 0.f;
        for (int k = 0; k < RPI; ++k) a += red[(k * CG + g) * 8 + j];
        y[(long)n * C + c] = f2bf(a * inv);
    }
}

__global__ void __launch_bounds__(NT) avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                         int N, int HW, int C) {
    const int CG = C >> 3;
    const long total = (long)N * HW * CG;
    const float inv = 1.f / HW;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        const int cg = (int)(i % CG);
        const long np = i / CG;
        const int n = (int)(np / HW);
        float g[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(dy + (long)n * C + cg * 8), g);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] *= inv;
        *reinterpret_cast<u16x8_t*>(dx + np * C + cg * 8) = pack8(g);
    }
}
}  // namespace

PDNN_API int pdnn_maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho,
                              int Wo, int k, int st, int pad, hipStream_t s) {
    const long work = (long)N * Ho * Wo * (C / 8);
    if ((long)N * H * W * C >= (1L << 31)) return 2;      // 32-bit index math in the kernels
    if (k == 3)
        hipLaunchKernelGGL(maxpool_fwd_kernel<3>, dim3(stream_grid(work, NT)), dim3(NT), 0, s, x, y, idx, N, H, W,
                           C, Ho, Wo, k, st, pad);
    else
        hipLaunchKernelGGL(maxpool_fwd_kernel<0>, dim3(stream_grid(work, NT)), dim3(NT), 0, s, x, y, idx, N, H, W,
                           C, Ho, Wo, k, st, pad);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                              int Ho, int Wo, int k, int st, int pad, hipStream_t s) {
    const long work = (long)N * H * W * (C / 8);
    if ((long)N * H * W * C >= (1L << 31)) return 2;      // 32-bit index math in the kernels
    if (k == 3 && st == 2)
        hipLaunchKernelGGL((maxpool_bwd_kernel<3, 2>), dim3(stream_grid(work, NT)), dim3(NT), 0, s, dy, idx, dx, N, H, W,
                           C, Ho, Wo, k, st, pad);
    else
        hipLaunchKernelGGL((maxpool_bwd_kernel<0, 0>), dim3(stream_grid(work, NT)), dim3(NT), 0, s, dy, idx, dx, N, H, W,
                           C, Ho, Wo, k, st, pad);
    PDNN_LAUNCH_RET;
}

// partial rows of the fused stem max-pool backward's BN slab ([rows][2][C] floats); 0 = shape unsupported
PDNN_API int pdnn_maxpool_bwd_bnred_rows(int N, int Ho, int Wo, int C) {
    if (C % 8 || C > 2048 || NT % (C / 8)) return 0;
    if ((long)N * 4 * Ho * Wo * C >= (1L << 31)) return 0;
    const long work = (long)N * Ho * Wo * (C / 8);
    long g = (work + NT - 1) / NT;
    return (int)(g < 1 ? 1 : g > 512 ? 512 : g);         // one wave of blocks: 174 VGPRs = 2 blocks per CU
}

// dy [N][Ho][Wo][C], idx its window bytes, t [N][2Ho][2Wo][C] (pre-BN) -> dx (pooled gradient, same shape
// as t) + the mode-2 BN-backward slab (pdnn_maxpool_bwd_bnred_rows rows).  3x3 / s2 / p1 window only.
PDNN_API int pdnn_maxpool_bwd_bnred(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, const bf16_t* t,
                                    const float* mean, const float* invstd, const float* mscale,
                                    const float* mshift, float* slab, int N, int Ho, int Wo, int C,
                                    hipStream_t s) {
    const int rows = pdnn_maxpool_bwd_bnred_rows(N, Ho, Wo, C);
    if (!rows) return 2;
    hipLaunchKernelGGL(maxpool_bwd_bnred_kernel, dim3(rows), dim3(NT), 0, s, dy, idx, dx, t, mean, invstd, mscale,
                       mshift, slab, N, Ho, Wo, C);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t s) {
    hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(N), dim3(NT), 0, s, x, y, HW, C);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t s) {
    const long work = (long)N * HW * (C / 8);
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(stream_grid(work, NT)), dim3(NT), 0, s, dy, dx, N, HW, C);
    PDNN_LAUNCH_RET;
}
