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

PDNN_API int pdnn_avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t s) {
    hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(N), dim3(NT), 0, s, x, y, HW, C);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t s) {
    const long work = (long)N * HW * (C / 8);
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(stream_grid(work, NT)), dim3(NT), 0, s, dy, dx, N, HW, C);
    PDNN_LAUNCH_RET;
}
