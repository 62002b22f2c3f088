// FP8 (OCP e4m3fn, gfx950) support: per-tensor quantisation with amax tracking, and the lane-layout probe
// of the block-scaled MFMA `v_mfma_scale_f32_16x16x128_f8f6f4` (SURVEY.md §2.8 K-18 "fp8 GEMM with
// per-tensor scaling"; BASELINE.json config 5).  The fp8 GEMM itself is the glds engine of gemm_mfma.hip
// instantiated for fp8 operands (DT = 1).
#include "common.h"

namespace {
constexpr int NT = 256;
constexpr float FP8_MAX = 448.f;     // e4m3fn
constexpr int FP8_AMAX_PARTS = 1024;  // per-block amax partials of a delayed-scaling quantisation (quant grid cap)

typedef __attribute__((ext_vector_type(8))) int v8i;

// 8 floats -> 8 e4m3 bytes (2 dwords), saturating
__device__ __forceinline__ uint2 f32x8_to_fp8(const float* v) {
    int w0 = 0, w1 = 0;
    float c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fminf(fmaxf(v[j], -FP8_MAX), FP8_MAX);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[0], c[1], w0, false);
    w0 = __builtin_amdgcn_cvt_pk_fp8_f32(c[2], c[3], w0, true);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[4], c[5], w1, false);
    w1 = __builtin_amdgcn_cvt_pk_fp8_f32(c[6], c[7], w1, true);
    return make_uint2((uint32_t)w0, (uint32_t)w1);
}

// amax of |x| (bf16, n % 8 == 0) -> atomicMax into *amax (float bits of a non-negative value order as uint)
__global__ void __launch_bounds__(NT) amax_bf16_kernel(const bf16_t* __restrict__ x, long n8, float* amax) {
    float m = 0.f;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float v[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(x + 8 * i), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    }
    m = wave_max(m);
    __shared__ float sm[NT / 64];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = sm[0];
        for (int i = 1; i < NT / 64; ++i) t = fmaxf(t, sm[i]);
        atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(t));
    }
}

// scale = FP8_MAX / amax * 2^-margin (1 if amax == 0); inv = 1 / scale
__global__ void fp8_scale_kernel(const float* amax, float* scale, float* inv, int margin) {
    const float a = *amax;
    const float s = a > 0.f ? ldexpf(FP8_MAX / a, -margin) : 1.f;
    *scale = s;
    *inv = 1.f / s;
}

// Delayed-scaling bookkeeping of one fp8 GEMM input, run right after its quantisation:
// gemm_scale = inv (the inverse scale the tensor was just quantised with) * inv_w; then the next call's
// scale is derived from the amax recorded by that quantisation, and the amax accumulator is reset.
__global__ void __launch_bounds__(NT) fp8_scale_step_kernel(float* amax, float* scale, float* inv, const float* inv_w,
                                                            float* gemm_scale, int margin, float fmax) {
    // amax holds FP8_AMAX_PARTS per-block partial maxima of the last quantisation (quant_fp8_kernel)
    float m = 0.f;
    for (int i = threadIdx.x; i < FP8_AMAX_PARTS; i += NT) {
        m = fmaxf(m, amax[i]);
        amax[i] = 0.f;
    }
    m = wave_max(m);
    __shared__ float sm[NT / 64];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = sm[0];
        for (int i = 1; i < NT / 64; ++i) a = fmaxf(a, sm[i]);
        if (gemm_scale) gemm_scale[0] = inv[0] * (inv_w ? inv_w[0] : 1.f);
        if (a > 0.f) {
            const float s = ldexpf(fmax / a, -margin);
            scale[0] = s;
            inv[0] = 1.f / s;
        }
    }
}

// out = e4m3(x * scale[0]), optionally also tracking amax of x (for the next step's delayed scale)
__global__ void __launch_bounds__(NT) quant_fp8_kernel(const bf16_t* __restrict__ x, long n8,
                                                       const float* __restrict__ scale, uint8_t* __restrict__ out,
                                                       float* amax) {
    const float s = *scale;
    float m = 0.f;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float v[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(x + 8 * i), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            m = fmaxf(m, fabsf(v[j]));
            v[j] *= s;
        }
        *reinterpret_cast<uint2*>(out + 8 * i) = f32x8_to_fp8(v);
    }
    if (amax) {      // one partial per block (no same-address atomics: 8k of them serialised this kernel)
        m = wave_max(m);
        __shared__ float sm[NT / 64];
        if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {
            float t = sm[0];
            for (int i = 1; i < NT / 64; ++i) t = fmaxf(t, sm[i]);
            amax[blockIdx.x] = fmaxf(amax[blockIdx.x], t);
        }
    }
}

// Current scaling in two launches and no fill: amax_parts_kernel writes one partial max per block of a fixed
// FP8_AMAX_PARTS-block grid (every entry overwritten); quant_fp8_cur_kernel reduces the partials in every
// block, quantises with scale = FP8_MAX / amax * 2^-margin and block 0 stores inv = 1 / scale.
__global__ void __launch_bounds__(NT) amax_parts_kernel(const bf16_t* __restrict__ x, long n8, float* __restrict__ parts) {
    float m = 0.f;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float v[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(x + 8 * i), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(v[j]));
    }
    m = wave_max(m);
    __shared__ float sm[NT / 64];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = sm[0];
        for (int i = 1; i < NT / 64; ++i) t = fmaxf(t, sm[i]);
        parts[blockIdx.x] = t;
    }
}

__global__ void __launch_bounds__(NT) quant_fp8_cur_kernel(const bf16_t* __restrict__ x, long n8,
                                                           const float* __restrict__ parts, uint8_t* __restrict__ out,
                                                           float* __restrict__ inv, int margin) {
    float m = 0.f;
    for (int i = threadIdx.x; i < FP8_AMAX_PARTS; i += NT) m = fmaxf(m, parts[i]);
    m = wave_max(m);
    __shared__ float sm[NT / 64];
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    float a = sm[0];
    for (int i = 1; i < NT / 64; ++i) a = fmaxf(a, sm[i]);
    const float s = a > 0.f ? ldexpf(FP8_MAX / a, -margin) : 1.f;
    if (blockIdx.x == 0 && threadIdx.x == 0) inv[0] = 1.f / s;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float v[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(x + 8 * i), v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= s;
        *reinterpret_cast<uint2*>(out + 8 * i) = f32x8_to_fp8(v);
    }
}

// fp32 master weights -> e4m3 with the given scale (the optimizer's fp8 weight shadow)
__global__ void __launch_bounds__(NT) quant_fp8_f32_kernel(const float* __restrict__ x, long n8,
                                                           const float* __restrict__ scale, uint8_t* __restrict__ out) {
    const float s = *scale;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        const float4 a = *reinterpret_cast<const float4*>(x + 8 * i);
        const float4 b = *reinterpret_cast<const float4*>(x + 8 * i + 4);
        float v[8] = {a.x * s, a.y * s, a.z * s, a.w * s, b.x * s, b.y * s, b.z * s, b.w * s};
        *reinterpret_cast<uint2*>(out + 8 * i) = f32x8_to_fp8(v);
    }
}

__global__ void __launch_bounds__(NT) amax_f32_kernel(const float* __restrict__ x, long n, float* amax) {
    float m = 0.f;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) m = fmaxf(m, fabsf(x[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(amax), __float_as_uint(m));
}

// e4m3 -> bf16 (dequantised with inv scale)
__global__ void __launch_bounds__(NT) dequant_fp8_kernel(const uint8_t* __restrict__ q, long n8,
                                                         const float* __restrict__ inv, bf16_t* __restrict__ out) {
    const float s = *inv;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        const uint2 w = *reinterpret_cast<const uint2*>(q + 8 * i);
        float v[8];
        v[0] = __builtin_amdgcn_cvt_f32_fp8((int)w.x, 0) * s;
        v[1] = __builtin_amdgcn_cvt_f32_fp8((int)w.x, 1) * s;
        v[2] = __builtin_amdgcn_cvt_f32_fp8((int)w.x, 2) * s;
        v[3] = __builtin_amdgcn_cvt_f32_fp8((int)w.x, 3) * s;
        v[4] = __builtin_amdgcn_cvt_f32_fp8((int)w.y, 0) * s;
        v[5] = __builtin_amdgcn_cvt_f32_fp8((int)w.y, 1) * s;
        v[6] = __builtin_amdgcn_cvt_f32_fp8((int)w.y, 2) * s;
        v[7] = __builtin_amdgcn_cvt_f32_fp8((int)w.y, 3) * s;
        *reinterpret_cast<u16x8_t*>(out + 8 * i) = pack8(v);
    }
}

// Layout probe of the block-scaled 16x16x128 MFMA with fp8 operands and unit block scales:
// layout 0: lane l holds A[l & 15][32 * (l >> 4) + e], e = 0..31 (and B[k][l & 15] likewise)
// layout 1: lane l holds k = 8 * (l >> 4) + (e & 7) + 32 * (e >> 3)
// A is [16][128] bytes (row = i), Bt is [16][128] bytes (row = j, B^T); D[i][j] fp32 [16][16].
__global__ void fp8_probe_kernel(const uint8_t* A, const uint8_t* Bt, float* D, int layout) {
    const int l = threadIdx.x, g = l >> 4, r = l & 15;
    v8i a, b;
#pragma unroll
    for (int d = 0; d < 8; ++d) {
        uint32_t wa = 0, wb = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = 4 * d + q;
            const int k = layout == 0 ? 32 * g + e : 8 * g + (e & 7) + 32 * (e >> 3);
            wa |= (uint32_t)A[r * 128 + k] << (8 * q);
            wb |= (uint32_t)Bt[r * 128 + k] << (8 * q);
        }
        a[d] = (int)wa;
        b[d] = (int)wb;
    }
    typedef __attribute__((ext_vector_type(4))) float v4f;
    v4f c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
#pragma unroll
    for (int q = 0; q < 4; ++q) D[(4 * g + q) * 16 + r] = c[q];
}
}  // namespace

PDNN_API int pdnn_fp8_probe(const uint8_t* A, const uint8_t* Bt, float* D, int layout, hipStream_t st) {
    hipLaunchKernelGGL(fp8_probe_kernel, dim3(1), dim3(64), 0, st, A, Bt, D, layout);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_amax_bf16(const bf16_t* x, long n, float* amax, hipStream_t st) {
    if (n % 8) return (int)hipErrorInvalidValue;
    unsigned g = stream_grid(n / 8, NT);
    if (g > 256) g = 256;            // one same-address atomic per block: keep them few
    hipLaunchKernelGGL(amax_bf16_kernel, dim3(g), dim3(NT), 0, st, x, n / 8, amax);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_amax_f32(const float* x, long n, float* amax, hipStream_t st) {
    hipLaunchKernelGGL(amax_f32_kernel, dim3(stream_grid(n, NT)), dim3(NT), 0, st, x, n, amax);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_fp8_scale(const float* amax, float* scale, float* inv, int margin, hipStream_t st) {
    hipLaunchKernelGGL(fp8_scale_kernel, dim3(1), dim3(1), 0, st, amax, scale, inv, margin);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_fp8_scale_step(float* amax, float* scale, float* inv, const float* inv_w, float* gemm_scale,
                                 int margin, hipStream_t st) {
    hipLaunchKernelGGL(fp8_scale_step_kernel, dim3(1), dim3(NT), 0, st, amax, scale, inv, inv_w, gemm_scale, margin,
                       FP8_MAX);
    PDNN_LAUNCH_RET;
}

// After a kernel that quantised in-line (the fp8 halo conv): reduce and reset the amax partials and roll the
// delayed scale forward (scale = fmax / amax * 2^-margin; e4m3 448, e5m2 57344).
PDNN_API int pdnn_fp8_scale_roll(float* amax, float* scale, float* inv, int e5m2, int margin, hipStream_t st) {
    hipLaunchKernelGGL(fp8_scale_step_kernel, dim3(1), dim3(NT), 0, st, amax, scale, inv, (const float*)nullptr,
                       (float*)nullptr, margin, e5m2 ? 57344.f : FP8_MAX);
    PDNN_LAUNCH_RET;
}

// amax (optional): FP8_AMAX_PARTS floats of per-block partial maxima (max-accumulated; reduced and reset by
// pdnn_fp8_scale_step)
PDNN_API int pdnn_quant_fp8(const bf16_t* x, long n, const float* scale, uint8_t* out, float* amax, hipStream_t st) {
    if (n % 8) return (int)hipErrorInvalidValue;
    unsigned g = stream_grid(n / 8, NT);
    if (g > FP8_AMAX_PARTS) g = FP8_AMAX_PARTS;
    hipLaunchKernelGGL(quant_fp8_kernel, dim3(g), dim3(NT), 0, st, x, n / 8, scale, out, amax);
    PDNN_LAUNCH_RET;
}

// out = e4m3(x * s), s from the tensor's own amax (current scaling), inv[0] = 1 / s; parts: FP8_AMAX_PARTS
// floats of workspace
PDNN_API int pdnn_quant_fp8_current(const bf16_t* x, long n, float* parts, uint8_t* out, float* inv, int margin,
                                    hipStream_t st) {
    if (n % 8) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(amax_parts_kernel, dim3(FP8_AMAX_PARTS), dim3(NT), 0, st, x, n / 8, parts);
    hipLaunchKernelGGL(quant_fp8_cur_kernel, dim3(FP8_AMAX_PARTS), dim3(NT), 0, st, x, n / 8, (const float*)parts,
                       out, inv, margin);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_quant_fp8_f32(const float* x, long n, const float* scale, uint8_t* out, hipStream_t st) {
    if (n % 8) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(quant_fp8_f32_kernel, dim3(stream_grid(n / 8, NT)), dim3(NT), 0, st, x, n / 8, scale, out);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_dequant_fp8(const uint8_t* q, long n, const float* inv, bf16_t* out, hipStream_t st) {
    if (n % 8) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(dequant_fp8_kernel, dim3(stream_grid(n / 8, NT)), dim3(NT), 0, st, q, n / 8, inv, out);
    PDNN_LAUNCH_RET;
}
