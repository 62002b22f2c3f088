// Fused optimizers and gradient-bucket kernels over FLAT fp32 buffers
// (SURVEY.md §2.8 K-13 gradient accumulate, K-14 average + SGD/Adam update, K-15 bucket
// flatten/scale; reference: pytorch_code/sync_replicas_master_nn.py:22-28,212-219 (avg + SGD),
// MPI_code/src/distributed/sync_replicas_master_nn.h:124-128 (ApplyGrad(lr/count)),
// distributed_TF/src/distributed_train.py:160 (Adam), data_parallel_dist.py:247-263 (flatten, /=world)).
//
// The framework keeps every parameter of a model in ONE contiguous fp32 master buffer and every
// gradient in one contiguous fp32 buffer (DDP buckets are views into it), so an optimizer step is a
// single launch over millions of elements instead of a per-tensor loop.  The same pass refreshes the
// bf16 compute shadow of the weights that the MFMA kernels read, and folds the gradient averaging
// factor (1/world, or 1/alive-count for k-of-n straggler mode) in as `gscale` read from device memory.
#include "common.h"

//
// Graph replay: a captured hipGraph bakes kernel arguments in, so the per-step hyper-parameters that
// change between replays (learning rate, Adam's bias corrections) can instead be read from a small
// device buffer `hyper` that the host refreshes (stream-ordered H2D copy) before each replay:
//   SGD:  hyper[0] = lr               Adam: hyper[0] = lr, hyper[1] = 1 - b1^t, hyper[2] = 1 - b2^t
// hyper == nullptr keeps the by-value arguments (eager mode).
namespace {
constexpr int NT = 256;

__global__ void __launch_bounds__(NT) sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                 float* __restrict__ buf, bf16_t* __restrict__ shadow, long n,
                                                 float lr, float momentum, float dampening, float wd,
                                                 int nesterov, const float* __restrict__ gscale_ptr,
                                                 float gscale, int first, const float* __restrict__ hyper) {
    const float gs = gscale_ptr ? gscale * (*gscale_ptr) : gscale;
    if (hyper) lr = hyper[0];
    const long n4 = n >> 2;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
        float4 pv = reinterpret_cast<float4*>(p)[i];
        const float4 gv = reinterpret_cast<const float4*>(g)[i];
        float pa[4] = {pv.x, pv.y, pv.z, pv.w};
        const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
        float ba[4] = {0, 0, 0, 0};
        if (momentum != 0.f && !first) {
            const float4 bv = reinterpret_cast<float4*>(buf)[i];
            ba[0] = bv.x; ba[1] = bv.y; ba[2] = bv.z; ba[3] = bv.w;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float d = ga[j] * gs + wd * pa[j];
            if (momentum != 0.f) {
                ba[j] = first ? d : momentum * ba[j] + (1.f - dampening) * d;
                d = nesterov ? d + momentum * ba[j] : ba[j];
            }
            pa[j] -= lr * d;
        }
        reinterpret_cast<float4*>(p)[i] = make_float4(pa[0], pa[1], pa[2], pa[3]);
        if (momentum != 0.f) reinterpret_cast<float4*>(buf)[i] = make_float4(ba[0], ba[1], ba[2], ba[3]);
        if (shadow) {
            u16x4_t s = {f2bf(pa[0]), f2bf(pa[1]), f2bf(pa[2]), f2bf(pa[3])};
            reinterpret_cast<u16x4_t*>(shadow)[i] = s;
        }
    }
    // tail
    for (long i = n4 * 4 + (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
        float d = g[i] * gs + wd * p[i];
        if (momentum != 0.f) {
            const float b = first ? d : momentum * buf[i] + (1.f - dampening) * d;
            buf[i] = b;
            d = nesterov ? d + momentum * b : b;
        }
        p[i] -= lr * d;
        if (shadow) shadow[i] = f2bf(p[i]);
    }
}

// Adam / AdamW (decoupled=1).  bc1 = 1 - beta1^t, bc2 = 1 - beta2^t (by value, or hyper[1..2]).
// Memory bound (16 B read + 14 B written per parameter): float4 loads/stores over the 16-B aligned
// body (`vec`, checked by the launcher), scalar tail.
struct AdamCoef {
    float lr, b1, b2, eps, wd, step, rbc2, gs;
    int decoupled;
    __device__ __forceinline__ void upd(float& pi, float gi, float& mi, float& vi) const {
        gi *= gs;
        if (decoupled) pi -= lr * wd * pi;
        else gi += wd * pi;
        mi = b1 * mi + (1.f - b1) * gi;
        vi = b2 * vi + (1.f - b2) * gi * gi;
        pi -= step * mi / (sqrtf(vi) * rbc2 + eps);
    }
};

__global__ void __launch_bounds__(NT) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  bf16_t* __restrict__ shadow, long n, float lr, float b1,
                                                  float b2, float eps, float wd, int decoupled, float bc1,
                                                  float bc2, const float* __restrict__ gscale_ptr,
                                                  float gscale, const float* __restrict__ hyper, int vec) {
    if (hyper) {
        lr = hyper[0];
        bc1 = hyper[1];
        bc2 = hyper[2];
    }
    const AdamCoef c{lr, b1, b2, eps, wd, lr / bc1, rsqrtf(bc2), gscale_ptr ? gscale * (*gscale_ptr) : gscale,
                     decoupled};
    const long n4 = vec ? (n >> 2) : 0;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n4; i += (long)gridDim.x * NT) {
        float4 pv = reinterpret_cast<float4*>(p)[i];
        const float4 gv = reinterpret_cast<const float4*>(g)[i];
        float4 mv = reinterpret_cast<float4*>(m)[i];
        float4 vv = reinterpret_cast<float4*>(v)[i];
        c.upd(pv.x, gv.x, mv.x, vv.x);
        c.upd(pv.y, gv.y, mv.y, vv.y);
        c.upd(pv.z, gv.z, mv.z, vv.z);
        c.upd(pv.w, gv.w, mv.w, vv.w);
        reinterpret_cast<float4*>(p)[i] = pv;
        reinterpret_cast<float4*>(m)[i] = mv;
        reinterpret_cast<float4*>(v)[i] = vv;
        if (shadow) {
            u16x4_t s = {f2bf(pv.x), f2bf(pv.y), f2bf(pv.z), f2bf(pv.w)};
            reinterpret_cast<u16x4_t*>(shadow)[i] = s;
        }
    }
    for (long i = n4 * 4 + (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
        float pi = p[i], mi = m[i], vi = v[i];
        c.upd(pi, g[i], mi, vi);
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
        if (shadow) shadow[i] = f2bf(pi);
    }
}

__global__ void __launch_bounds__(NT) cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                           long n, float scale) {
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) y[i] = f2bf(x[i] * scale);
}
__global__ void __launch_bounds__(NT) cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y,
                                                           long n, float scale, int accumulate) {
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) {
        const float v = bf2f(x[i]) * scale;
        y[i] = accumulate ? y[i] + v : v;
    }
}
__global__ void __launch_bounds__(NT) scale_f32_kernel(float* __restrict__ x, long n, float scale,
                                                       const float* __restrict__ dev_scale, int invert) {
    float s = scale;
    if (dev_scale) s *= invert ? 1.f / fmaxf(*dev_scale, 1.f) : *dev_scale;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) x[i] *= s;
}
// y += a * x  (fp32), used for gradient accumulation of the k-of-n alive-weighted contributions
__global__ void __launch_bounds__(NT) axpy_f32_kernel(float* __restrict__ y, const float* __restrict__ x, long n,
                                                      float a) {
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) y[i] += a * x[i];
}
// sum of squares (for grad-norm clipping / NaN checks): per-block partial into out[blockIdx]
__global__ void __launch_bounds__(NT) sumsq_kernel(const float* __restrict__ x, long n, float* __restrict__ out) {
    __shared__ float red[NT / 64];
    float s = 0.f;
    for (long i = (long)blockIdx.x * NT + threadIdx.x; i < n; i += (long)gridDim.x * NT) s += x[i] * x[i];
    s = block_sum<NT>(s, red);
    if (threadIdx.x == 0) atomicAdd(out, s);
}
}  // namespace

PDNN_API int pdnn_sgd_step(float* p, const float* g, float* buf, bf16_t* shadow, long n, float lr, float momentum,
                           float dampening, float wd, int nesterov, const float* gscale_ptr, float gscale, int first,
                           const float* hyper, hipStream_t st) {
    hipLaunchKernelGGL(sgd_kernel, dim3(stream_grid(n / 4 + 1, NT)), dim3(NT), 0, st, p, g, buf, shadow, n, lr,
                       momentum, dampening, wd, nesterov, gscale_ptr, gscale, first, hyper);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_adam_step(float* p, const float* g, float* m, float* v, bf16_t* shadow, long n, float lr, float b1,
                            float b2, float eps, float wd, int decoupled, float bc1, float bc2,
                            const float* gscale_ptr, float gscale, const float* hyper, hipStream_t st) {
    const uintptr_t a16 = reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) |
                          reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v);
    const int vec = (a16 & 15) == 0 && (reinterpret_cast<uintptr_t>(shadow) & 7) == 0;
    hipLaunchKernelGGL(adam_kernel, dim3(stream_grid(vec ? n / 4 + 1 : n, NT)), dim3(NT), 0, st, p, g, m, v, shadow,
                       n, lr, b1, b2, eps, wd, decoupled, bc1, bc2, gscale_ptr, gscale, hyper, vec);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_cast_f32_bf16(const float* x, bf16_t* y, long n, float scale, hipStream_t st) {
    hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(stream_grid(n, NT)), dim3(NT), 0, st, x, y, n, scale);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_cast_bf16_f32(const bf16_t* x, float* y, long n, float scale, int accumulate, hipStream_t st) {
    hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(stream_grid(n, NT)), dim3(NT), 0, st, x, y, n, scale, accumulate);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_scale_f32(float* x, long n, float scale, const float* dev_scale, int invert, hipStream_t st) {
    hipLaunchKernelGGL(scale_f32_kernel, dim3(stream_grid(n, NT)), dim3(NT), 0, st, x, n, scale, dev_scale, invert);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_axpy_f32(float* y, const float* x, long n, float a, hipStream_t st) {
    hipLaunchKernelGGL(axpy_f32_kernel, dim3(stream_grid(n, NT)), dim3(NT), 0, st, y, x, n, a);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_sumsq_f32(const float* x, long n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(sumsq_kernel, dim3(stream_grid(n, NT) > 512 ? 512 : stream_grid(n, NT)), dim3(NT), 0, st, x, n,
                       out);
    PDNN_LAUNCH_RET;
}
