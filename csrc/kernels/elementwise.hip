// Elementwise kernels (SURVEY.md §2.8 K-06 ReLU, K-07 residual add, K-10 sigmoid + derivative,
// K-17 input preprocessing, K-18 GELU).  All vectorised 16 bytes per lane (Guideline 13).
// Reference call sites: MPI_code/src/util/util.h:84-123 (Relu/Sigmoid and their gradients),
// pytorch_code/model_ops/resnet.py:32-35 (relu, residual add), pure_py_code/nn/nn_utils.py:4-8.
#include "common.h"

namespace {
constexpr int NT = 256;

// op: 0 relu, 1 sigmoid, 2 gelu(tanh), 3 identity
__device__ __forceinline__ float act_f(float x, int op) {
    if (op == 0) return fmaxf(x, 0.f);
    if (op == 1) return 1.f / (1.f + __expf(-x));
    if (op == 2) {
        const float k0 = 0.7978845608028654f, k1 = 0.044715f;
        return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
    }
    return x;
}
// derivative given the INPUT x (relu/gelu) or the OUTPUT y (sigmoid, y(1-y) as in util.h:115-123)
__device__ __forceinline__ float act_d(float x, int op) {
    if (op == 0) return x > 0.f ? 1.f : 0.f;
    if (op == 1) { const float y = 1.f / (1.f + __expf(-x)); return y * (1.f - y); }
    if (op == 2) {
        const float k0 = 0.7978845608028654f, k1 = 0.044715f;
        const float u = k0 * (x + k1 * x * x * x);
        const float t = tanhf(u);
        return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
    }
    return 1.f;
}

__global__ void __launch_bounds__(NT) act_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long n8,
                                                     int op) {
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float v[8];
        unpack8(reinterpret_cast<const u16x8_t*>(x)[i], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = act_f(v[j], op);
        reinterpret_cast<u16x8_t*>(y)[i] = pack8(v);
    }
}
__global__ void __launch_bounds__(NT) act_bwd_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ x,
                                                     bf16_t* __restrict__ dx, long n8, int op) {
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float gv[8], xv[8];
        unpack8(reinterpret_cast<const u16x8_t*>(g)[i], gv);
        unpack8(reinterpret_cast<const u16x8_t*>(x)[i], xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] *= act_d(xv[j], op);
        reinterpret_cast<u16x8_t*>(dx)[i] = pack8(gv);
    }
}
// y = a*alpha + b*beta (bf16)
__global__ void __launch_bounds__(NT) add_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                 bf16_t* __restrict__ y, long n8, float alpha, float beta) {
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long)gridDim.x * NT) {
        float av[8], bv[8];
        unpack8(reinterpret_cast<const u16x8_t*>(a)[i], av);
        unpack8(reinterpret_cast<const u16x8_t*>(b)[i], bv);
#pragma unroll
        for (int j = 0; j < 8; ++j) av[j] = av[j] * alpha + bv[j] * beta;
        reinterpret_cast<u16x8_t*>(y)[i] = pack8(av);
    }
}
// NCHW (fp32 or bf16) -> NHWC bf16 with the channel dim zero-padded to Cp (stem input, K-17).
// One thread per pixel; reads are coalesced along the pixel index, each group of 8 output channels is
// one 16-byte store (Cp % 8 == 0, checked on the host), index math in 32 bits per image.
template <typename T>
__global__ void __launch_bounds__(NT) nchw_to_nhwc_kernel(const T* __restrict__ x, bf16_t* __restrict__ y, int N,
                                                          int C, int HW, int Cp) {
    const long total = (long)N * HW;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        const int n = (int)(i / HW), p = (int)(i - (long)n * HW);
        const T* xs = x + (long)n * C * HW + p;
        for (int c0 = 0; c0 < Cp; c0 += 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = c0 + j < C ? Ld<T>::get(xs, (long)(c0 + j) * HW) : 0.f;
            *reinterpret_cast<u16x8_t*>(y + i * Cp + c0) = pack8(v);
        }
    }
}
// NHWC bf16 (channels Cp) -> NCHW fp32 gradient of the first C channels
__global__ void __launch_bounds__(NT) nhwc_to_nchw_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y,
                                                              int N, int C, int HW, int Cp) {
    const long total = (long)N * C * HW;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        const long p = i % HW, nc = i / HW, c = nc % C, n = nc / C;
        y[i] = bf2f(x[(n * HW + p) * Cp + c]);
    }
}
// column sums of a [rows][cols] bf16 matrix into fp32 (bias gradient of a Linear, K-03 fused column sum)
__global__ void __launch_bounds__(NT) colsum_kernel(const bf16_t* __restrict__ x, long rows, int cols,
                                                    float* __restrict__ out, int accumulate) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63);
    const int rq = threadIdx.x >> 6;
    __shared__ float red[4][64];
    float s = 0.f;
    if (c < cols)
        for (long r = rq; r < rows; r += 4) s += bf2f(x[r * cols + c]);
    red[rq][threadIdx.x & 63] = s;
    __syncthreads();
    if (rq == 0 && c < cols) {
        const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        out[c] = accumulate ? out[c] + t : t;
    }
}

// Two-level column sum for tall matrices (cols % 8 == 0): level 1 — block (column group of 512, row split
// y) accumulates 8 columns per lane over its rows with 16-byte loads and writes one partial row;
// level 2 sums the partial rows (deterministic, no atomics).  Sized so level 1 fills the chip (>= ~256
// blocks even for 768 columns: up to 128 row splits of >= 64 rows) and level 2 is a short unrolled
// reduction spread over 64-column blocks (bias gradients of a GPT-2 step are 60+ of these calls).
// ATOMIC: the block's sums are added straight into the output (no partial rows, no level-2 launch): for an
// accumulating destination (a bias gradient in the zero-initialised flat arena); fp32 add order varies.
template <bool ATOMIC>
__global__ void __launch_bounds__(NT) colsum_partial_kernel(const bf16_t* __restrict__ x, long rows, int cols,
                                                            float* __restrict__ part) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = (blockIdx.x * 64 + lane) * 8;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (c < cols) {
        const long r0 = (long)blockIdx.y * 4 + w, rs = (long)gridDim.y * 4;
        long r = r0;
        for (; r + rs < rows; r += 2 * rs) {          // two rows in flight per lane
            float v[8], u[8];
            unpack8(*reinterpret_cast<const u16x8_t*>(x + r * cols + c), v);
            unpack8(*reinterpret_cast<const u16x8_t*>(x + (r + rs) * cols + c), u);
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += v[j] + u[j];
        }
        if (r < rows) {
            float v[8];
            unpack8(*reinterpret_cast<const u16x8_t*>(x + r * cols + c), v);
#pragma unroll
            for (int j = 0; j < 8; ++j) s[j] += v[j];
        }
    }
    __shared__ float red[4][512];
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = s[j];
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += NT) {
        const int cc = blockIdx.x * 512 + i;
        if (cc < cols) {
            const float t = red[0][i] + red[1][i] + red[2][i] + red[3][i];
            if (ATOMIC) atomicAdd(part + cc, t);
            else part[(long)blockIdx.y * cols + cc] = t;
        }
    }
}

// level 2: block = 64 columns x 4 row groups, 4 independent accumulators per lane
__global__ void __launch_bounds__(NT) colsum_final_kernel(const float* __restrict__ part, int nrows, int cols,
                                                          float* __restrict__ out, int accumulate) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if (c < cols) {
        int r = w;
        for (; r + 12 < nrows; r += 16) {
            a0 += part[(long)r * cols + c];
            a1 += part[(long)(r + 4) * cols + c];
            a2 += part[(long)(r + 8) * cols + c];
            a3 += part[(long)(r + 12) * cols + c];
        }
        for (; r < nrows; r += 4) a0 += part[(long)r * cols + c];
    }
    __shared__ float red[4][64];
    red[w][lane] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (w == 0 && c < cols) {
        const float t = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
        out[c] = accumulate ? out[c] + t : t;
    }
}
// y[n][i][j][:] = x[n][st*i][st*j][:] (NHWC bf16, C % 8 == 0): the pixels a 1x1 / stride-st / pad-0 conv reads,
// made contiguous so that conv runs as a plain stride-1 1x1 conv (A-stationary / ping-pong engines) and its weight
// gradient as a plain GEMM (the ResNet shortcut convs; fused_resnet.py).  One thread per 16-byte chunk, a run of
// C/8 consecutive threads per pixel: each pixel's channels are one contiguous 2*C-byte read.
__global__ void __launch_bounds__(NT) subsample_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int H,
                                                       int W, int C, int Ho, int Wo, int st, long total) {
    const int C8 = C >> 3;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
        const long pix = i / C8;
        const int c = (int)(i - pix * C8) * 8;
        const long nh = pix / Wo;
        const int j = (int)(pix - nh * Wo);
        const long n = nh / Ho;
        const int h = (int)(nh - n * Ho);
        const long src = ((n * H + (long)st * h) * W + (long)st * j) * C + c;
        *reinterpret_cast<u16x8_t*>(y + pix * C + c) = *reinterpret_cast<const u16x8_t*>(x + src);
    }
}

}  // namespace

PDNN_API int pdnn_colsum_splits(long rows) {
    const long s = rows / 64;                    // >= 64 rows (16 per wave) per split, at most 128 splits
    return (int)(s < 1 ? 1 : (s > 128 ? 128 : s));
}

PDNN_API int pdnn_act_fwd(const bf16_t* x, bf16_t* y, long n, int op, hipStream_t st) {
    hipLaunchKernelGGL(act_fwd_kernel, dim3(stream_grid(n / 8, NT)), dim3(NT), 0, st, x, y, n / 8, op);
    PDNN_LAUNCH_RET;
}
PDNN_API int pdnn_act_bwd(const bf16_t* g, const bf16_t* x, bf16_t* dx, long n, int op, hipStream_t st) {
    hipLaunchKernelGGL(act_bwd_kernel, dim3(stream_grid(n / 8, NT)), dim3(NT), 0, st, g, x, dx, n / 8, op);
    PDNN_LAUNCH_RET;
}
PDNN_API int pdnn_add(const bf16_t* a, const bf16_t* b, bf16_t* y, long n, float alpha, float beta, hipStream_t st) {
    hipLaunchKernelGGL(add_kernel, dim3(stream_grid(n / 8, NT)), dim3(NT), 0, st, a, b, y, n / 8, alpha, beta);
    PDNN_LAUNCH_RET;
}
PDNN_API int pdnn_nchw_to_nhwc(const void* x, int x_bf16, bf16_t* y, int N, int C, int HW, int Cp, hipStream_t st) {
    if (Cp % 8 != 0 || C > Cp) return 1;                 // hipErrorInvalidValue: 16-byte channel groups
    if (x_bf16)
        hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, dim3(stream_grid((long)N * HW, NT)), dim3(NT), 0, st,
                           (const bf16_t*)x, y, N, C, HW, Cp);
    else
        hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(stream_grid((long)N * HW, NT)), dim3(NT), 0, st,
                           (const float*)x, y, N, C, HW, Cp);
    PDNN_LAUNCH_RET;
}
PDNN_API int pdnn_nhwc_to_nchw_f32(const bf16_t* x, float* y, int N, int C, int HW, int Cp, hipStream_t st) {
    hipLaunchKernelGGL(nhwc_to_nchw_f32_kernel, dim3(stream_grid((long)N * C * HW, NT)), dim3(NT), 0, st, x, y, N, C,
                       HW, Cp);
    PDNN_LAUNCH_RET;
}
// work: pdnn_colsum_splits(rows) * cols floats for the two-level deterministic form (cols % 8 == 0, rows > 256);
// accumulate with no work: the one-launch atomic form for those shapes
PDNN_API int pdnn_colsum(const bf16_t* x, long rows, int cols, float* out, int accumulate, float* work,
                         hipStream_t st) {
    if (accumulate && !work && cols % 8 == 0 && rows > 256) {
        hipLaunchKernelGGL(colsum_partial_kernel<true>, dim3((cols + 511) / 512, pdnn_colsum_splits(rows)), dim3(NT), 0,
                           st, x, rows, cols, out);
    } else if (work && cols % 8 == 0 && rows > 256) {
        const int sp = pdnn_colsum_splits(rows);
        hipLaunchKernelGGL(colsum_partial_kernel<false>, dim3((cols + 511) / 512, sp), dim3(NT), 0, st, x, rows, cols, work);
        hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 63) / 64), dim3(NT), 0, st, work, sp, cols, out,
                           accumulate);
    } else {
        hipLaunchKernelGGL(colsum_kernel, dim3((cols + 63) / 64), dim3(NT), 0, st, x, rows, cols, out, accumulate);
    }
    PDNN_LAUNCH_RET;
}

// ------------------------------------------------------------------------------------------------
// bf16 matrix transpose dst[c][r] = src[r][c] (row strides lds / ldd): 64 x 64 tiles through LDS,
// 16-byte global loads and stores (8 bf16 per lane), LDS rows padded by 2 elements (odd word stride)
// so the column reads of the transposed pass hit distinct banks.  Used for the reduction-major copies of
// the transformer weights (ops/functional.weight_bf16_t): the data-gradient GEMM then reads K-major B.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void transpose_tile(const bf16_t* __restrict__ src, long lds, bf16_t* __restrict__ dst,
                                               long ldd, int R, int C, int r0, int c0, bf16_t (*t)[66]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 2; ++i) {                     // 64 rows x 8 chunks = 512 loads
        const int k = tid + 256 * i, rr = k >> 3, cc = (k & 7) * 8;
        const int r = r0 + rr, c = c0 + cc;
        u16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (r < R && c + 8 <= C) v = *reinterpret_cast<const u16x8_t*>(src + (long)r * lds + c);
        else if (r < R) for (int j = 0; j < 8 && c + j < C; ++j) v[j] = src[(long)r * lds + c + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[rr][cc + j] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int k = tid + 256 * i, cr = k >> 3, rc = (k & 7) * 8;    // output row = source column
        const int c = c0 + cr, r = r0 + rc;
        if (c >= C) continue;
        u16x8_t v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = t[rc + j][cr];
        if (r + 8 <= R) *reinterpret_cast<u16x8_t*>(dst + (long)c * ldd + r) = v;
        else for (int j = 0; j < 8 && r + j < R; ++j) dst[(long)c * ldd + r + j] = v[j];
    }
}

__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16_t* __restrict__ src, long lds, bf16_t* __restrict__ dst,
                                                             long ldd, int R, int C) {
    __shared__ bf16_t t[64][66];
    transpose_tile(src, lds, dst, ldd, R, C, blockIdx.y * 64, blockIdx.x * 64, t);
}

// W'[c][8 - tap][k] = W[k][tap][c]: the tap-flipped transposed 3x3 weight of the data gradients (conv3x3.hip, conv_s2.hip)
// as nine 64 x 64-tiled transposes in one launch (blockIdx.z = tap).  The element-wise flip took 25 us a call at
// ResNet-50 stage 4 on the forward's side stream (r6_03 trace: 11 calls, 0.27 ms per step).
__global__ void __launch_bounds__(256) conv3x3_flip_tiled_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                                                 int K, int C) {
    __shared__ bf16_t t[64][66];
    const int tap = blockIdx.z;
    transpose_tile(w + (long)tap * C, 9L * C, wt + (long)(8 - tap) * K, 9L * K, K, C, blockIdx.y * 64, blockIdx.x * 64, t);
}

// Many contiguous matrices in one launch (the transposed weight copies of a whole transformer, refreshed
// once per optimizer step instead of one ~5 us launch per weight inside the backward).  The table rides in
// the kernel arguments; block b belongs to the last entry with tile0 <= b (binary search, scalar loads).
constexpr int TMULTI = 64;
struct TDesc {
    const bf16_t* src;
    bf16_t* dst;
    int R, C, tiles_c, tile0;
};
struct TBatch {
    TDesc d[TMULTI];
    int n;
};
__global__ void __launch_bounds__(256) transpose_bf16_multi_kernel(const TBatch b) {
    __shared__ bf16_t t[64][66];
    const int blk = blockIdx.x;
    int lo = 0, hi = b.n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (b.d[mid].tile0 <= blk) lo = mid;
        else hi = mid - 1;
    }
    const TDesc& e = b.d[lo];
    const int k = blk - e.tile0, tr = k / e.tiles_c, tc = k - tr * e.tiles_c;
    transpose_tile(e.src, e.C, e.dst, e.R, e.R, e.C, tr * 64, tc * 64, t);
}

PDNN_API int pdnn_transpose_bf16(const bf16_t* src, long lds, bf16_t* dst, long ldd, int R, int C, hipStream_t st) {
    hipLaunchKernelGGL(transpose_bf16_kernel, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, st, src, lds, dst, ldd, R, C);
    PDNN_LAUNCH_RET;
}
// srcs[i] [R[i]][C[i]] (contiguous) -> dsts[i] [C[i]][R[i]]; any count (launches of TMULTI matrices each)
PDNN_API int pdnn_transpose_bf16_multi(const bf16_t* const* srcs, bf16_t* const* dsts, const int* R, const int* C,
                                       int n, hipStream_t st) {
    for (int base = 0; base < n; base += TMULTI) {
        TBatch b;
        b.n = n - base < TMULTI ? n - base : TMULTI;
        int tiles = 0;
        for (int i = 0; i < b.n; ++i) {
            const int q = base + i;
            if (R[q] <= 0 || C[q] <= 0) return 1;        // hipErrorInvalidValue
            b.d[i] = TDesc{srcs[q], dsts[q], R[q], C[q], (C[q] + 63) / 64, tiles};
            tiles += ((R[q] + 63) / 64) * ((C[q] + 63) / 64);
        }
        hipLaunchKernelGGL(transpose_bf16_multi_kernel, dim3(tiles), dim3(256), 0, st, b);
        const int e = (int)hipGetLastError();
        if (e) return e;
    }
    return 0;
}

// y = x[:, ::st, ::st, :] (NHWC bf16): Ho = (H - 1) / st + 1, Wo likewise; C % 8 == 0
PDNN_API int pdnn_subsample(const bf16_t* x, bf16_t* y, int N, int H, int W, int C, int st, hipStream_t s) {
    if (C % 8 || st < 1 || N < 1 || H < 1 || W < 1) return (int)hipErrorInvalidValue;
    const int Ho = (H - 1) / st + 1, Wo = (W - 1) / st + 1;
    const long total = (long)N * Ho * Wo * (C / 8);
    long g = (total + NT - 1) / NT;
    if (g > 2048) g = 2048;        // a pure copy: 8 blocks per CU of grid-stride threads keep enough loads in flight
    hipLaunchKernelGGL(subsample_kernel, dim3((unsigned)g), dim3(NT), 0, s, x, y, H, W, C, Ho, Wo, st, total);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_conv3x3_flip_tiled(const bf16_t* w, bf16_t* wt, int K, int C, hipStream_t st) {
    if (K < 1 || C < 1) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(conv3x3_flip_tiled_kernel, dim3((C + 63) / 64, (K + 63) / 64, 9), dim3(256), 0, st, w, wt, K, C);
    PDNN_LAUNCH_RET;
}
