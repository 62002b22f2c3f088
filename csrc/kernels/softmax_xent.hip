// Fused softmax + cross-entropy (reference: nn.CrossEntropyLoss in
// pytorch_code/distributed_worker.py:86,161, MPI_code/src/util/util.h:125-144 Softmax/LogDot,
// MPI_code/src/nn/nn_layer.h:150-152 fused (p - onehot) gradient).
//
// Forward: one pass over each logits row with an online (max, sum-exp) pair per lane, merged across the
// block -> per-row loss = lse - x[label] and the row's log-sum-exp saved for backward.
// Backward: one more pass writing dlogits = (softmax - onehot) * scale, scale = grad_out / rows read from
// a DEVICE pointer (no host sync; graph-capturable).  Rows with label == ignore_index get zero grad.
// Works for 10-class heads and the 50257-way GPT-2 vocabulary alike; bf16 rows whose length and stride
// are multiples of 8 take 16-byte vector loads/stores (the 50304-padded GPT-2 head: HBM-speed passes).
#include "common.h"

namespace {
constexpr int NT = 256;

template <typename T>
__device__ __forceinline__ void online(float& m, float& s, float v) {
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
}

template <typename T, bool VEC>
__global__ void __launch_bounds__(NT) xent_fwd_kernel(const T* __restrict__ logits, long ld, int V,
                                                      const int64_t* __restrict__ labels, int ignore,
                                                      float* __restrict__ loss, float* __restrict__ lse,
                                                      float* __restrict__ loss_sum, float* __restrict__ count) {
    const long row = blockIdx.x;
    const T* x = logits + row * ld;
    float m = -INFINITY, s = 0.f;
    if (VEC) {
        // 16-byte loads (8 bf16 per lane), one rescale per chunk: the row is read at HBM speed
        const u16x8_t* x8 = reinterpret_cast<const u16x8_t*>(x);
        const int n8 = V / 8;
        for (int i = threadIdx.x; i < n8; i += 2 * NT) {       // two 16-byte loads in flight per lane
            const bool two = i + NT < n8;
            const u16x8_t a = x8[i];
            const u16x8_t b = two ? x8[i + NT] : a;
            float v[16];
            unpack8(a, v);
            unpack8(b, v + 8);
            float cm = v[0];
#pragma unroll
            for (int j = 1; j < 16; ++j) cm = fmaxf(cm, v[j]);
            if (cm > m) {
                s = (m == -INFINITY) ? 0.f : s * __expf(m - cm);
                m = cm;
            }
            float t = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) t += __expf(v[j] - m);
            if (two) {
#pragma unroll
                for (int j = 8; j < 16; ++j) t += __expf(v[j] - m);
            }
            s += t;
        }
    } else {
        for (int i = threadIdx.x; i < V; i += NT) online<T>(m, s, Ld<T>::get(x, i));
    }
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

template <typename T, bool VEC>
__global__ void __launch_bounds__(NT) xent_bwd_kernel(const T* __restrict__ logits, long ld, int V,
                                                      const int64_t* __restrict__ labels, int ignore,
                                                      const float* __restrict__ lse,
                                                      const float* __restrict__ gscale, float denom,
                                                      const float* __restrict__ count,
                                                      T* __restrict__ dlogits, long ldd) {
    const long row = blockIdx.x;
    const T* x = logits + row * ld;
    T* d = dlogits + row * ldd;
    const int64_t y = labels[row];
    const bool ign = (y == ignore || y < 0 || y >= V);
    // count (optional): the forward's device-side count of non-ignored rows (mean reduction), so the caller
    // needs no scalar kernels to form g / max(count, 1)
    const float sc = ign ? 0.f : (*gscale) / (count ? fmaxf(*count, 1.f) : denom);
    const float l = lse[row];
    if (VEC) {
        const u16x8_t* x8 = reinterpret_cast<const u16x8_t*>(x);
        u16x8_t* d8 = reinterpret_cast<u16x8_t*>(d);
        const int n8 = V / 8;
        for (int i = threadIdx.x; i < n8; i += 2 * NT) {       // two 16-byte loads in flight per lane
            const bool two = i + NT < n8;
            const u16x8_t a = x8[i];
            const u16x8_t b = two ? x8[i + NT] : a;
            float v[8], u[8];
            unpack8(a, v);
            unpack8(b, u);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                v[j] = sc * (__expf(v[j] - l) - (8 * i + j == y ? 1.f : 0.f));
                u[j] = sc * (__expf(u[j] - l) - (8 * (i + NT) + j == y ? 1.f : 0.f));
            }
            d8[i] = pack8(v);
            if (two) d8[i + NT] = pack8(u);
        }
        return;
    }
    for (int i = threadIdx.x; i < V; i += NT) {
        const float p = __expf(Ld<T>::get(x, i) - l);
        Ld<T>::put(d, i, sc * (p - (i == y ? 1.f : 0.f)));
    }
}
// Training forward that also writes the UNSCALED gradient softmax - onehot (bf16, in place over the logits allowed):
// the row is held in registers (MAXC 16-byte chunks per lane, V <= 8 * NT * MAXC), so it is read from HBM once
// and written once -- the separate backward pass (a second full read of the logits) disappears.  The caller
// applies grad_out / count to the products of the gradient (the LM head's 8192 x 768 operands), not to it.
template <int MAXC>
__global__ void __launch_bounds__(NT) xent_fwd_grad_kernel(const bf16_t* __restrict__ logits, long ld, int V,
                                                           const int64_t* __restrict__ labels, int ignore,
                                                           float* __restrict__ loss, float* __restrict__ lse,
                                                           bf16_t* dlogits, long ldd) {
    __shared__ float red[NT / 64];
    const long row = blockIdx.x;
    const u16x8_t* x8 = reinterpret_cast<const u16x8_t*>(logits + row * ld);
    u16x8_t* d8 = reinterpret_cast<u16x8_t*>(dlogits + row * ldd);
    const int n8 = V / 8;
    u16x8_t r[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int i = threadIdx.x + c * NT;
        if (i < n8) r[c] = x8[i];
    }
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int i = threadIdx.x + c * NT;
        if (i < n8) {
            float v[8];
            unpack8(r[c], v);
#pragma unroll
            for (int j = 0; j < 8; ++j) mx = fmaxf(mx, v[j]);
        }
    }
    mx = wave_max(mx);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = mx;
    __syncthreads();
    float M = red[0];
#pragma unroll
    for (int k = 1; k < NT / 64; ++k) M = fmaxf(M, red[k]);
    __syncthreads();
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int i = threadIdx.x + c * NT;
        if (i < n8) {
            float v[8];
            unpack8(r[c], v);
#pragma unroll
            for (int j = 0; j < 8; ++j) sum += __expf(v[j] - M);
        }
    }
    const float l = M + __logf(block_sum<NT>(sum, red));
    const int64_t y = labels[row];
    const bool ign = (y == ignore || y < 0 || y >= V);
    if (threadIdx.x == 0) {
        lse[row] = l;
        loss[row] = ign ? 0.f : l - bf2f(logits[row * ld + y]);
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int i = threadIdx.x + c * NT;
        if (i < n8) {
            float v[8];
            unpack8(r[c], v);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ign ? 0.f : __expf(v[j] - l) - (8 * i + j == y ? 1.f : 0.f);
            d8[i] = pack8(v);
        }
    }
}
}  // namespace

// dtype: 0 = fp32 logits, 1 = bf16 logits
namespace {
// loss_sum[0] = sum of the per-row losses, count[0] = rows with a valid label (one block, no atomics)
__global__ void __launch_bounds__(1024) xent_sum_kernel(const float* __restrict__ loss, const int64_t* __restrict__ labels,
                                                        int rows, int V, int ignore, float* __restrict__ loss_sum,
                                                        float* __restrict__ count) {
    float s = 0.f, c = 0.f;
    for (int r = threadIdx.x; r < rows; r += 1024) {
        const int64_t y = labels[r];
        s += loss[r];
        c += (y == ignore || y < 0 || y >= V) ? 0.f : 1.f;
    }
    s = wave_sum(s);
    c = wave_sum(c);
    __shared__ float ps[16], pc[16];
    if ((threadIdx.x & 63) == 0) { ps[threadIdx.x >> 6] = s; pc[threadIdx.x >> 6] = c; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float S = 0.f, Cn = 0.f;
        for (int i = 0; i < 16; ++i) { S += ps[i]; Cn += pc[i]; }
        loss_sum[0] = S;
        if (count) count[0] = Cn;
    }
}
}  // namespace

// loss_sum / count (optional): SET to the loss sum and the valid-label count by a second one-block kernel over the
// per-row losses (8192 same-address atomics from the row blocks cost 123 us of a 264 us GPT-2 head forward, r4_49)
PDNN_API int pdnn_xent_fwd(const void* logits, long ld, int rows, int V, const int64_t* labels, int ignore,
                           float* loss, float* lse, float* loss_sum, float* count, int dtype, hipStream_t st) {
    if (loss_sum && !loss) return (int)hipErrorInvalidValue;
    float* const lsum = loss_sum;
    float* const cnt = count;
    loss_sum = nullptr;                          // the row kernels take no atomics
    count = nullptr;
    const bool vec = dtype == 1 && V % 8 == 0 && ld % 8 == 0 && (reinterpret_cast<uintptr_t>(logits) & 15) == 0;
    if (vec)
        hipLaunchKernelGGL((xent_fwd_kernel<bf16_t, true>), dim3(rows), dim3(NT), 0, st, (const bf16_t*)logits, ld,
                           V, labels, ignore, loss, lse, loss_sum, count);
    else if (dtype == 1)
        hipLaunchKernelGGL((xent_fwd_kernel<bf16_t, false>), dim3(rows), dim3(NT), 0, st, (const bf16_t*)logits, ld,
                           V, labels, ignore, loss, lse, loss_sum, count);
    else
        hipLaunchKernelGGL((xent_fwd_kernel<float, false>), dim3(rows), dim3(NT), 0, st, (const float*)logits, ld, V,
                           labels, ignore, loss, lse, loss_sum, count);
    if (lsum)
        hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(1024), 0, st, (const float*)loss, labels, rows, V, ignore, lsum,
                           cnt);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_xent_bwd(const void* logits, long ld, int rows, int V, const int64_t* labels, int ignore,
                           const float* lse, const float* gscale, float denom, const float* count, void* dlogits,
                           long ldd, int dtype, hipStream_t st) {
    const bool vec = dtype == 1 && V % 8 == 0 && ld % 8 == 0 && ldd % 8 == 0 &&
                     ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(dlogits)) & 15) == 0;
    if (vec)
        hipLaunchKernelGGL((xent_bwd_kernel<bf16_t, true>), dim3(rows), dim3(NT), 0, st, (const bf16_t*)logits, ld,
                           V, labels, ignore, lse, gscale, denom, count, (bf16_t*)dlogits, ldd);
    else if (dtype == 1)
        hipLaunchKernelGGL((xent_bwd_kernel<bf16_t, false>), dim3(rows), dim3(NT), 0, st, (const bf16_t*)logits, ld,
                           V, labels, ignore, lse, gscale, denom, count, (bf16_t*)dlogits, ldd);
    else
        hipLaunchKernelGGL((xent_bwd_kernel<float, false>), dim3(rows), dim3(NT), 0, st, (const float*)logits, ld,
                           V, labels, ignore, lse, gscale, denom, count, (float*)dlogits, ldd);
    PDNN_LAUNCH_RET;
}

// bf16 logits [rows][ld] (V % 8 == 0, ld % 8 == 0, ldd % 8 == 0, 16-byte aligned, V <= 51200) -> per-row loss / lse,
// loss_sum / count SET as in pdnn_xent_fwd, and dlogits = softmax - onehot UNSCALED (dlogits == logits allowed).
PDNN_API int pdnn_xent_fwd_grad(const bf16_t* logits, long ld, int rows, int V, const int64_t* labels, int ignore,
                                float* loss, float* lse, float* loss_sum, float* count, bf16_t* dlogits, long ldd,
                                hipStream_t st) {
    constexpr int MAXC = 25;
    if (V % 8 || ld % 8 || ldd % 8 || V > 8 * NT * MAXC || !loss || !lse ||
        ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(dlogits)) & 15))
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(xent_fwd_grad_kernel<MAXC>, dim3(rows), dim3(NT), 0, st, logits, ld, V, labels, ignore, loss, lse,
                       dlogits, ldd);
    if (loss_sum)
        hipLaunchKernelGGL(xent_sum_kernel, dim3(1), dim3(1024), 0, st, (const float*)loss, labels, rows, V, ignore,
                           loss_sum, count);
    PDNN_LAUNCH_RET;
}
