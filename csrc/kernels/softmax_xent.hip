// Fused softmax + cross-entropy (reference: nn.CrossEntropyLoss in
// pytorch_code/distributed_worker.py:86,161, MPI_code/src/util/util.h:125-144 Softmax/LogDot,
// MPI_code/src/nn/nn_layer.h:150-152 fused (p - onehot) gradient).
//
// Forward: one pass over each logits row with an online (max, sum-exp) pair per lane, merged across the
// block -> per-row loss = lse - x[label] and the row's log-sum-exp saved for backward.
// Backward: one more pass writing dlogits = (softmax - onehot) * scale, scale = grad_out / rows read from
// a DEVICE pointer (no host sync; graph-capturable).  Rows with label == ignore_index get zero grad.
// Works for 10-class heads and the 50257-way GPT-2 vocabulary alike (16-byte vector loads for bf16).
#include "common.h"

namespace {
constexpr int NT = 256;

template <typename T>
__device__ __forceinline__ void online(float& m, float& s, float v) {
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
}

template <typename T>
__global__ void __launch_bounds__(NT) xent_fwd_kernel(const T* __restrict__ logits, long ld, int V,
                                                      const int64_t* __restrict__ labels, int ignore,
                                                      float* __restrict__ loss, float* __restrict__ lse,
                                                      float* __restrict__ loss_sum, float* __restrict__ count) {
    const long row = blockIdx.x;
    const T* x = logits + row * ld;
    float m = -INFINITY, s = 0.f;
    for (int i = threadIdx.x; i < V; i += NT) online<T>(m, s, Ld<T>::get(x, i));
    // merge (m, s) across the block
    __shared__ float sm[NT / 64], ss[NT / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
        const float mm = fmaxf(m, m2);
        s = (m == -INFINITY ? 0.f : s * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
        m = mm;
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = sm[0], S = ss[0];
        for (int i = 1; i < NT / 64; ++i) {
            const float mm = fmaxf(M, sm[i]);
            S = S * __expf(M - mm) + ss[i] * __expf(sm[i] - mm);
            M = mm;
        }
        const float l = M + __logf(S);
        lse[row] = l;
        const int64_t y = labels[row];
        const float li = (y == ignore || y < 0 || y >= V) ? 0.f : (l - Ld<T>::get(x, (long)y));
        if (loss) loss[row] = li;
        if (loss_sum) {
            atomicAdd(loss_sum, li);
            if (count && !(y == ignore || y < 0 || y >= V)) atomicAdd(count, 1.f);
        }
    }
}

template <typename T>
__global__ void __launch_bounds__(NT) xent_bwd_kernel(const T* __restrict__ logits, long ld, int V,
                                                      const int64_t* __restrict__ labels, int ignore,
                                                      const float* __restrict__ lse,
                                                      const float* __restrict__ gscale, float denom,
                                                      T* __restrict__ dlogits, long ldd) {
    const long row = blockIdx.x;
    const T* x = logits + row * ld;
    T* d = dlogits + row * ldd;
    const int64_t y = labels[row];
    const bool ign = (y == ignore || y < 0 || y >= V);
    const float sc = ign ? 0.f : (*gscale) / denom;
    const float l = lse[row];
    for (int i = threadIdx.x; i < V; i += NT) {
        const float p = __expf(Ld<T>::get(x, i) - l);
        Ld<T>::put(d, i, sc * (p - (i == y ? 1.f : 0.f)));
    }
}
}  // namespace

// dtype: 0 = fp32 logits, 1 = bf16 logits
PDNN_API int pdnn_xent_fwd(const void* logits, long ld, int rows, int V, const int64_t* labels, int ignore,
                           float* loss, float* lse, float* loss_sum, float* count, int dtype, hipStream_t st) {
    if (dtype == 1)
        hipLaunchKernelGGL(xent_fwd_kernel<bf16_t>, dim3(rows), dim3(NT), 0, st, (const bf16_t*)logits, ld, V,
                           labels, ignore, loss, lse, loss_sum, count);
    else
        hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(rows), dim3(NT), 0, st, (const float*)logits, ld, V,
                           labels, ignore, loss, lse, loss_sum, count);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_xent_bwd(const void* logits, long ld, int rows, int V, const int64_t* labels, int ignore,
                           const float* lse, const float* gscale, float denom, void* dlogits, long ldd, int dtype,
                           hipStream_t st) {
    if (dtype == 1)
        hipLaunchKernelGGL(xent_bwd_kernel<bf16_t>, dim3(rows), dim3(NT), 0, st, (const bf16_t*)logits, ld, V,
                           labels, ignore, lse, gscale, denom, (bf16_t*)dlogits, ldd);
    else
        hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(rows), dim3(NT), 0, st, (const float*)logits, ld, V,
                           labels, ignore, lse, gscale, denom, (float*)dlogits, ldd);
    PDNN_LAUNCH_RET;
}
