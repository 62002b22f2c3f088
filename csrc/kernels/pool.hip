// Pooling kernels, NHWC bf16 (SURVEY.md §2.8 K-08 MaxPool, K-09 AvgPool;
// reference call sites pytorch_code/model_ops/lenet.py:22-25, resnet.py:94).
//
// Max pool saves the winning window position as one byte per output element so the backward is a
// gather (each input position visits the <= ceil(k/s)^2 windows that cover it) — no atomics, and
// deterministic even with overlapping 3x3/s2 windows.
#include "common.h"

namespace {
constexpr int NT = 256;

__global__ void __launch_bounds__(NT) maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                         int Ho, int Wo, int k, int st, int pad) {
    const int CG = C >> 3;
    const long total = (long)N * Ho * Wo * CG;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        long t = i;
        const int cg = (int)(t % CG); t /= CG;
        const int wo = (int)(t % Wo); t /= Wo;
        const int ho = (int)(t % Ho);
        const int n = (int)(t / Ho);
        float best[8];
        uint8_t bi[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; }
        for (int r = 0; r < k; ++r) {
            const int hi = ho * st - pad + r;
            if ((unsigned)hi >= (unsigned)H) continue;
            for (int s = 0; s < k; ++s) {
                const int wi = wo * st - pad + s;
                if ((unsigned)wi >= (unsigned)W) continue;
                float v[8];
                unpack8(*reinterpret_cast<const u16x8_t*>(x + (((long)n * H + hi) * W + wi) * C + cg * 8), v);
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (v[j] > best[j] || (v[j] != v[j])) { best[j] = v[j]; bi[j] = (uint8_t)(r * k + s); }
            }
        }
        const long o = (((long)n * Ho + ho) * Wo + wo) * C + cg * 8;
        *reinterpret_cast<u16x8_t*>(y + o) = pack8(best);
        if (idx) {
            uint2 packed;
            packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
            packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
            *reinterpret_cast<uint2*>(idx + o) = packed;
        }
    }
}

__global__ void __launch_bounds__(NT) maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                         const uint8_t* __restrict__ idx,
                                                         bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                         int Ho, int Wo, int k, int st, int pad) {
    const int CG = C >> 3;
    const long total = (long)N * H * W * CG;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        long t = i;
        const int cg = (int)(t % CG); t /= CG;
        const int w = (int)(t % W); t /= W;
        const int h = (int)(t % H);
        const int n = (int)(t / H);
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        // outputs ho with ho*st - pad <= h <= ho*st - pad + k - 1
        const int ho_lo = max(0, (h + pad - k + st) / st), ho_hi = min(Ho - 1, (h + pad) / st);
        const int wo_lo = max(0, (w + pad - k + st) / st), wo_hi = min(Wo - 1, (w + pad) / st);
        for (int ho = ho_lo; ho <= ho_hi; ++ho) {
            const int r = h + pad - ho * st;
            if (r < 0 || r >= k) continue;
            for (int wo = wo_lo; wo <= wo_hi; ++wo) {
                const int s = w + pad - wo * st;
                if (s < 0 || s >= k) continue;
                const long o = (((long)n * Ho + ho) * Wo + wo) * C + cg * 8;
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
        *reinterpret_cast<u16x8_t*>(dx + (((long)n * H + h) * W + w) * C + cg * 8) = pack8(acc);
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
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(stream_grid(work, NT)), dim3(NT), 0, s, x, y, idx, N, H, W, C,
                       Ho, Wo, k, st, pad);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                              int Ho, int Wo, int k, int st, int pad, hipStream_t s) {
    const long work = (long)N * H * W * (C / 8);
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(stream_grid(work, NT)), dim3(NT), 0, s, dy, idx, dx, N, H, W, C,
                       Ho, Wo, k, st, pad);
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
