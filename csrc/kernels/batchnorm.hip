// BatchNorm2d (training + eval) for NHWC bf16 activations with fp32 statistics (SURVEY.md §2.8 K-05,
// K-06, K-07; reference modules: pytorch_code/model_ops/resnet.py:20-35, 45-63).
//
// The statistics pass is normally FUSED into the producing convolution's epilogue
// (gemm_mfma.hip writes per-64-row partial (sum, sumsq) slabs); `pdnn_bn_stats` is the standalone
// version for inputs that were not produced by our conv.  The normalisation itself is usually fused
// into the CONSUMING convolution's operand loader (affine + ReLU prologue), so the only materialising
// kernel in a ResNet block is `pdnn_bn_apply` at the block output, which also fuses the residual
// branch (identity, or the downsample conv's own BN) and the final ReLU.
//
// Slab layout shared by every partial-statistics producer: [rows][2][C] fp32 — for partial row i,
// slab[(2i)*C + c] = sum, slab[(2i+1)*C + c] = sum of squares (or, in backward, sum(g) / sum(g*xhat)).
//
// Memory layout: x is [L][C] with L = N*H*W, channel fastest.  Each thread owns 8 consecutive channels
// (16-byte loads, Guideline 13); C must be a multiple of 8 and C/8 <= 256.
#include "common.h"

namespace {
constexpr int NT = 256;

// Rows per thread per iteration of the streaming kernels: all U rows' loads are issued before any is
// consumed.  Measured on the ResNet-50 bs256 step (gpu_run44 / gpu_run45 in dev/gpu_runs/archive_r1_r3.txt), img/s:
// U=2 everywhere 7530-7556, U=4 7508, U=8 7400 (VGPR pressure costs more occupancy than the extra loads
// in flight buy); reduce U=1/2/4 and 16 vs 64 rows per thread-row all within noise; apply U=1 7553.
// The templated reduce kernel itself (mode / second-BN specialisations) was the +2% (7385 -> 7530+).
// The apply kernels are software-pipelined across rows instead (next row's loads before this row's stores).
// A/B builds override the reduce unroll with -DPDNN_BN_UR=n.
#ifndef PDNN_BN_UR
#define PDNN_BN_UR 2
#endif
// Minimum rows per thread-row of a statistics reduction (more blocks for the narrow, short late layers:
// ResNet-50 layer4 has only 12544 rows of 2048 channels at bs256); 32 with the 512-block cap of reduce_grid:
// ResNet-50 +1.0% over 64 / 1024 (profiles/resnet50_bn_grid_r4.txt, gpurun_out/r4_70-71)
#ifndef PDNN_BN_RMIN
#define PDNN_BN_RMIN 32
#endif
// wide-grid slab finalize (bn_slab_level1 + bn_slab_final); 0 = the older slab_reduce + finalize path
#ifndef PDNN_BN_WIDE_FIN
#define PDNN_BN_WIDE_FIN 1
#endif
constexpr int BN_UR = PDNN_BN_UR, BN_RMIN = PDNN_BN_RMIN;

// Level-1 reduction of a partial-statistics slab [rows][2][C] -> [RB][2][C]: block (cx, ry) sums the
// rows ry, ry+RB, ... for 64 channels with 4 row lanes (coalesced 256-byte row segments).
__global__ void __launch_bounds__(NT) slab_reduce_kernel(const float* __restrict__ slab, int rows, int C,
                                                          float* __restrict__ out) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), lr = threadIdx.x >> 6;
    const int RB = gridDim.y;
    __shared__ float red[2][4][64];
    float s = 0.f, q = 0.f;
    if (c < C) {
        for (int r = blockIdx.y + RB * lr; r < rows; r += RB * 4) {
            s += slab[(long)(2 * r) * C + c];
            q += slab[(long)(2 * r + 1) * C + c];
        }
    }
    red[0][lr][threadIdx.x & 63] = s;
    red[1][lr][threadIdx.x & 63] = q;
    __syncthreads();
    if (lr == 0 && c < C) {
        const int l = threadIdx.x;
        out[(long)(2 * blockIdx.y) * C + c] = red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l];
        out[(long)(2 * blockIdx.y + 1) * C + c] = red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l];
    }
}

// finalize (few) partial rows -> mean, invstd, scale/shift (+ running-stat update), fp64 accumulation.
// Block = 64 channels x 4 row-lanes (rows strided by 4, combined through LDS).
__global__ void __launch_bounds__(NT) bn_finalize_kernel(const float* __restrict__ slab, int rows, int C, double L,
                                                         float eps, float momentum, const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* run_mean,
                                                         float* run_var, float* mean_out, float* invstd_out,
                                                         float* scale_out, float* shift_out) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), lr = threadIdx.x >> 6;
    __shared__ double red[2][4][64];
    double s = 0.0, q = 0.0;
    if (c < C)
        for (int r = lr; r < rows; r += 4) {
            s += slab[(long)(2 * r) * C + c];
            q += slab[(long)(2 * r + 1) * C + c];
        }
    red[0][lr][threadIdx.x & 63] = s;
    red[1][lr][threadIdx.x & 63] = q;
    __syncthreads();
    if (lr != 0 || c >= C) return;
    const int l = threadIdx.x;
    s = red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l];
    q = red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l];
    const double mean = s / L;
    double var = q / L - mean * mean;
    if (var < 0) var = 0;
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
        const double unb = L > 1 ? var * L / (L - 1) : var;
        run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mean);
        run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
    }
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    if (mean_out) mean_out[c] = (float)mean;
    if (invstd_out) invstd_out[c] = inv;
    scale_out[c] = g * inv;
    shift_out[c] = b - (float)mean * g * inv;
}

// Statistics finalize of a slab [rows][2][C] in two launches: a level-1 pass over a wide grid (float4
// loads, 16 channel groups x 16 row lanes per block, RB blocks per 64-channel column) into `work`
// [RB][2][C], then one block per column sums the RB rows in fp64 and runs the epilogue.  The old level-1
// had only C/64 x 64 blocks of scalar loads (20 us for ResNet-50's 12544-row layer1 slabs).  A one-launch
// variant (last-arriving block finalizes) measured 3-8x slower per call: the agent-scope release fence
// every block needs writes back the XCD's whole L2 (buffer_wbl2) right after a conv epilogue filled it.
constexpr int FIN_RB_MAX = 256;       // level-1 rows per column (work holds FIN_RB_MAX * 2 * C floats)

struct FinFwd {
    double L; float eps, momentum;
    const float *gamma, *beta; float *run_mean, *run_var, *mean_out, *invstd_out, *scale_out, *shift_out;
    __device__ void operator()(int c, double s, double q) const {
        const double mean = s / L;
        double var = q / L - mean * mean;
        if (var < 0) var = 0;
        const float inv = (float)(1.0 / sqrt(var + (double)eps));
        if (run_mean) {
            const double unb = L > 1 ? var * L / (L - 1) : var;
            run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mean);
            run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
        }
        const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
        if (mean_out) mean_out[c] = (float)mean;
        if (invstd_out) invstd_out[c] = inv;
        scale_out[c] = g * inv;
        shift_out[c] = b - (float)mean * g * inv;
    }
};

struct FinBwd {
    float *dgamma, *dbeta; int accumulate; float *gacc, *bacc;
    __device__ void operator()(int c, double s, double q) const {
        if (accumulate) { dbeta[c] += (float)s; dgamma[c] += (float)q; }
        else { dbeta[c] = (float)s; dgamma[c] = (float)q; }
        if (gacc) { gacc[c] += (float)q; bacc[c] += (float)s; }     // direct accumulation into param grads
    }
};

__global__ void __launch_bounds__(NT) bn_slab_level1_kernel(const float* __restrict__ slab, int rows, int C,
                                                             float* __restrict__ work) {
    const int col = blockIdx.x, RB = gridDim.y, y = blockIdx.y;
    const int ch = threadIdx.x & 15, lane = threadIdx.x >> 4;
    const int c0 = col * 64 + ch * 4;
    const bool on = c0 < C;
    __shared__ float4 red[2][16][16];
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
    if (on) {
        const int stride = RB * 16;
        int r = y * 16 + lane;
        for (; r + stride < rows; r += 2 * stride) {       // two rows' loads in flight
            const float4 a0 = *reinterpret_cast<const float4*>(slab + (long)(2 * r) * C + c0);
            const float4 b0 = *reinterpret_cast<const float4*>(slab + (long)(2 * r + 1) * C + c0);
            const float4 a1 = *reinterpret_cast<const float4*>(slab + (long)(2 * (r + stride)) * C + c0);
            const float4 b1 = *reinterpret_cast<const float4*>(slab + (long)(2 * (r + stride) + 1) * C + c0);
            s.x += a0.x + a1.x; s.y += a0.y + a1.y; s.z += a0.z + a1.z; s.w += a0.w + a1.w;
            q.x += b0.x + b1.x; q.y += b0.y + b1.y; q.z += b0.z + b1.z; q.w += b0.w + b1.w;
        }
        if (r < rows) {
            const float4 a0 = *reinterpret_cast<const float4*>(slab + (long)(2 * r) * C + c0);
            const float4 b0 = *reinterpret_cast<const float4*>(slab + (long)(2 * r + 1) * C + c0);
            s.x += a0.x; s.y += a0.y; s.z += a0.z; s.w += a0.w;
            q.x += b0.x; q.y += b0.y; q.z += b0.z; q.w += b0.w;
        }
    }
    red[0][lane][ch] = s;
    red[1][lane][ch] = q;
    __syncthreads();
    if (lane == 0 && on) {
        float4 a = red[0][0][ch], b = red[1][0][ch];
        for (int k = 1; k < 16; ++k) {
            const float4 u = red[0][k][ch], v = red[1][k][ch];
            a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
            b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
        }
        *reinterpret_cast<float4*>(work + (long)(2 * y) * C + c0) = a;
        *reinterpret_cast<float4*>(work + (long)(2 * y + 1) * C + c0) = b;
    }
}

// level 2: block = one 64-channel column, 16 float4 channel groups x 16 row lanes, fp64 sums.
template <class Epi>
__global__ void __launch_bounds__(NT) bn_slab_final_kernel(const float* __restrict__ part, int rows, int C, Epi epi) {
    const int col = blockIdx.x, ch = threadIdx.x & 15, lane = threadIdx.x >> 4;
    const int c0 = col * 64 + ch * 4;
    double sd[4] = {0, 0, 0, 0}, qd[4] = {0, 0, 0, 0};
    if (c0 < C)
        for (int r = lane; r < rows; r += 16) {
            const float4 a = *reinterpret_cast<const float4*>(part + (long)(2 * r) * C + c0);
            const float4 b = *reinterpret_cast<const float4*>(part + (long)(2 * r + 1) * C + c0);
            sd[0] += a.x; sd[1] += a.y; sd[2] += a.z; sd[3] += a.w;
            qd[0] += b.x; qd[1] += b.y; qd[2] += b.z; qd[3] += b.w;
        }
    __shared__ double redd[2][16][64];
#pragma unroll
    for (int j = 0; j < 4; ++j) { redd[0][lane][ch * 4 + j] = sd[j]; redd[1][lane][ch * 4 + j] = qd[j]; }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int c = col * 64 + threadIdx.x;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) { a += redd[0][k][threadIdx.x]; b += redd[1][k][threadIdx.x]; }
        if (c < C) epi(c, a, b);
    }
}

// One-launch finalize: the level-1 blocks of a column hand their partial rows to the column's LAST-arriving
// block, which sums them and runs the epilogue (cdna_hip_programming.md §6 Guideline 16, counter form): the
// partial rows are stored write-through (sc1, so no release fence and no L2 write-back of the conv output
// that just filled it -- the cost that sank a __threadfence() version), the storing wave drains them
// (vmcnt(0)) before one lane draws a ticket with an agent-scope atomic, and the last arriver acquires once
// and reads the rows with sc1 loads.  `cnt` holds one zeroed counter per column; the last arriver puts it
// back to zero, so a pool of counters is reused across calls without a memset launch.
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ void st_sc1(float* p, float4 v) {     // 16 bytes as two 8-byte sc1 stores
    gu64* g = (gu64*)p;
    __hip_atomic_store(g, (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(g + 1, (unsigned long long)__float_as_uint(v.z) | ((unsigned long long)__float_as_uint(v.w) << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld_sc1(const float* p) {
    const gu64* g = (const gu64*)p;
    const unsigned long long lo = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long hi = __hip_atomic_load(g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float4(__uint_as_float((unsigned)lo), __uint_as_float((unsigned)(lo >> 32)),
                       __uint_as_float((unsigned)hi), __uint_as_float((unsigned)(hi >> 32)));
}

template <class Epi>
__global__ void __launch_bounds__(NT) bn_slab_fused_kernel(const float* __restrict__ slab, int rows, int C,
                                                           float* work, unsigned* cnt, Epi epi) {
    const int col = blockIdx.x, RB = gridDim.y, y = blockIdx.y;
    const int ch = threadIdx.x & 15, lane = threadIdx.x >> 4;
    const int c0 = col * 64 + ch * 4;
    const bool on = c0 < C;
    __shared__ double redd[2][16][64];
    float4* red = reinterpret_cast<float4*>(&redd[0][0][0]);    // level-1 view: [2][16][16] float4
    __shared__ int last;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f), q = s;
    if (on) {
        const int stride = RB * 16;
        int r = y * 16 + lane;
        for (; r + 3 * stride < rows; r += 4 * stride) {
            float4 a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = *reinterpret_cast<const float4*>(slab + (long)(2 * (r + j * stride)) * C + c0);
                b[j] = *reinterpret_cast<const float4*>(slab + (long)(2 * (r + j * stride) + 1) * C + c0);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                s.x += a[j].x; s.y += a[j].y; s.z += a[j].z; s.w += a[j].w;
                q.x += b[j].x; q.y += b[j].y; q.z += b[j].z; q.w += b[j].w;
            }
        }
        for (; r < rows; r += stride) {
            const float4 a0 = *reinterpret_cast<const float4*>(slab + (long)(2 * r) * C + c0);
            const float4 b0 = *reinterpret_cast<const float4*>(slab + (long)(2 * r + 1) * C + c0);
            s.x += a0.x; s.y += a0.y; s.z += a0.z; s.w += a0.w;
            q.x += b0.x; q.y += b0.y; q.z += b0.z; q.w += b0.w;
        }
    }
    red[lane * 16 + ch] = s;
    red[256 + lane * 16 + ch] = q;
    __syncthreads();
    if (threadIdx.x < 64) {                  // wave 0: lanes 0..15 publish this block's row, lane 0 draws the ticket
        if (lane == 0 && on) {
            float4 a = red[ch], b = red[256 + ch];
            for (int k = 1; k < 16; ++k) {
                const float4 u = red[k * 16 + ch], v = red[256 + k * 16 + ch];
                a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
                b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
            }
            st_sc1(work + (long)(2 * y) * C + c0, a);
            st_sc1(work + (long)(2 * y + 1) * C + c0, b);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // the storing wave drains its sc1 stores
        if (threadIdx.x == 0) {
            const unsigned t = __hip_atomic_fetch_add((gu32*)(cnt + col), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = t == (unsigned)(RB - 1);
        }
    }
    __syncthreads();                          // also: every wave is done with the level-1 LDS view
    if (!last) return;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    double sd[4] = {0, 0, 0, 0}, qd[4] = {0, 0, 0, 0};
    if (on) {
        int r = lane;
        for (; r + 48 < RB; r += 64) {
            float4 a[4], b[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = ld_sc1(work + (long)(2 * (r + 16 * j)) * C + c0);
                b[j] = ld_sc1(work + (long)(2 * (r + 16 * j) + 1) * C + c0);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                sd[0] += a[j].x; sd[1] += a[j].y; sd[2] += a[j].z; sd[3] += a[j].w;
                qd[0] += b[j].x; qd[1] += b[j].y; qd[2] += b[j].z; qd[3] += b[j].w;
            }
        }
        for (; r < RB; r += 16) {
            const float4 a = ld_sc1(work + (long)(2 * r) * C + c0);
            const float4 b = ld_sc1(work + (long)(2 * r + 1) * C + c0);
            sd[0] += a.x; sd[1] += a.y; sd[2] += a.z; sd[3] += a.w;
            qd[0] += b.x; qd[1] += b.y; qd[2] += b.z; qd[3] += b.w;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { redd[0][lane][ch * 4 + j] = sd[j]; redd[1][lane][ch * 4 + j] = qd[j]; }
    __syncthreads();
    if (threadIdx.x < 64) {
        const int c = col * 64 + threadIdx.x;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) { a += redd[0][k][threadIdx.x]; b += redd[1][k][threadIdx.x]; }
        if (c < C) epi(c, a, b);
        if (threadIdx.x == 0) __hip_atomic_store((gu32*)(cnt + col), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

inline unsigned fin_rows(int rows) {       // level-1 blocks per column: >= 4 slab rows per thread
    int rb = rows / (16 * 4);
    if (rows <= 64) return 0;                // few rows: level 2 reads the slab directly
    if (rb > FIN_RB_MAX) rb = FIN_RB_MAX;
    if (rb < 1) rb = 1;
    return (unsigned)rb;
}

// eval-mode scale/shift from running statistics
__global__ void bn_eval_coeff_kernel(int C, float eps, const float* gamma, const float* beta,
                                     const float* rm, const float* rv, float* scale, float* shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float inv = rsqrtf(rv[c] + eps);
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    scale[c] = g * inv;
    shift[c] = b - rm[c] * g * inv;
}

// Per-channel partial sum / sumsq over a grid-strided row range.
__global__ void __launch_bounds__(NT) bn_stats_kernel(const bf16_t* __restrict__ x, long L, int C,
                                                      float* __restrict__ slab) {
    __shared__ float red[2][NT * 8];
    const int CG = C >> 3;                 // channel groups of 8
    const int RPI = NT / CG;               // rows per iteration
    const int t = threadIdx.x, cg = t % CG, rr = t / CG;
    float s[8] = {0}, q[8] = {0};
    if (rr < RPI) {
        for (long r = (long)blockIdx.x * RPI + rr; r < L; r += (long)gridDim.x * RPI) {
            float v[8];
            unpack8(*reinterpret_cast<const u16x8_t*>(x + r * C + cg * 8), v);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s[j] += v[j]; q[j] += v[j] * v[j]; }
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { red[0][t * 8 + j] = s[j]; red[1][t * 8 + j] = q[j]; }
    __syncthreads();
    for (int c = t; c < C; c += NT) {
        const int g = c >> 3, j = c & 7;
        float a = 0.f, b = 0.f;
        for (int k = 0; k < RPI; ++k) { a += red[0][(k * CG + g) * 8 + j]; b += red[1][(k * CG + g) * 8 + j]; }
        slab[(long)(2 * blockIdx.x) * C + c] = a;
        slab[(long)(2 * blockIdx.x + 1) * C + c] = b;
    }
}

// y = act(x*scale + shift + residual'), residual' = res (identity) or res*rscale + rshift.
// Each thread owns one fixed group of 8 channels (coefficients in registers) and strides over rows.
// MASK: also write the sign bits of y (bit j of byte [row][c/8] = y[row][c + j] > 0, 1/16 of y's bytes), so
// the backward's ReLU mask (mask mode 3) does not re-read the whole bf16 output.
template <bool RES, bool RSC, bool RELU, bool MASK>
__global__ void __launch_bounds__(NT) bn_apply_kernel(const bf16_t* __restrict__ x, long L, int C,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift,
                                                      const bf16_t* __restrict__ res,
                                                      const float* __restrict__ rscale,
                                                      const float* __restrict__ rshift,
                                                      bf16_t* __restrict__ y, uint8_t* __restrict__ mbits) {
    const int CG = C >> 3, RPI = NT / CG;
    const int t = threadIdx.x, cg = t % CG, rr = t / CG, c = cg * 8;
    if (rr >= RPI) return;
    float sc[8], sh[8], rs_[RSC ? 8 : 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        sc[j] = scale[c + j];
        sh[j] = shift[c + j] + (RSC ? rshift[c + j] : 0.f);
        if constexpr (RSC) rs_[j] = rscale[c + j];
    }
    // Software-pipelined over the rows this thread visits: row r+step's operands are loaded BEFORE row r's
    // stores (s_waitcnt vmcnt counts stores too on gfx9: loads issued after a store wait for it, so the
    // load-then-store loop serialised one store drain + load latency per row), unconditionally from a clamped
    // row (the last row is re-read once, never stored twice).
    const long step = (long)gridDim.x * RPI;
    long r = (long)blockIdx.x * RPI + rr;
    if (r >= L) return;
    u16x8_t xv = *reinterpret_cast<const u16x8_t*>(x + r * C + c), rv;
    if constexpr (RES) rv = *reinterpret_cast<const u16x8_t*>(res + r * C + c);
    for (; r < L; r += step) {
        const long rn = r + step < L ? r + step : L - 1;
        const u16x8_t xn = *reinterpret_cast<const u16x8_t*>(x + rn * C + c);
        u16x8_t rnv;
        if constexpr (RES) rnv = *reinterpret_cast<const u16x8_t*>(res + rn * C + c);
        float v[8];
        unpack8(xv, v);
        if constexpr (RES) {
            float rf[8];
            unpack8(rv, rf);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], sc[j], fmaf(rf[j], RSC ? rs_[j] : 1.f, sh[j]));
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], sc[j], sh[j]);
        }
        if constexpr (RELU) {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
        }
        if constexpr (MASK) {
            unsigned bits = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) bits |= (v[j] > 0.f ? 1u : 0u) << j;
            mbits[r * CG + cg] = (uint8_t)bits;
        }
        *reinterpret_cast<u16x8_t*>(y + r * C + c) = pack8(v);
        xv = xn;
        if constexpr (RES) rv = rnv;
    }
}

// mask modes for the backward: 0 none, 1 mask = (msrc > 0), 2 mask = (x*mscale + mshift > 0),
// 3 mask = bit j of byte msrc[row][c/8] (written by bn_apply's MASK variant)
// partial sums of gm and gm*xhat (xhat = (x-mean)*invstd) for one or two BNs sharing gm.
// Specialised on the mask mode and the second BN so unused operands take no registers.
template <int MODE, bool X2>
__global__ void __launch_bounds__(NT) bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ x, long L, int C,
    const float* __restrict__ mean, const float* __restrict__ invstd,
    const bf16_t* __restrict__ msrc, const float* __restrict__ mscale, const float* __restrict__ mshift,
    float* __restrict__ slab, const bf16_t* __restrict__ x2, const float* __restrict__ mean2,
    const float* __restrict__ invstd2, float* __restrict__ slab2) {
    __shared__ float red[2][NT * 8];
    const int CG = C >> 3, RPI = NT / CG;
    const int t = threadIdx.x, cg = t % CG, rr = t / CG, c = cg * 8;
    float s[8] = {0}, q[8] = {0}, q2[X2 ? 8 : 1] = {0};
    float mu[8], is[8], mu2[X2 ? 8 : 1], is2[X2 ? 8 : 1], ms[MODE == 2 ? 8 : 1], mh[MODE == 2 ? 8 : 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        mu[j] = mean[c + j]; is[j] = invstd[c + j];
        if constexpr (X2) { mu2[j] = mean2[c + j]; is2[j] = invstd2[c + j]; }
        if constexpr (MODE == 2) { ms[j] = mscale[c + j]; mh[j] = mshift[c + j]; }
    }
    if (rr < RPI) {
        const long step = (long)gridDim.x * RPI;
        for (long r0 = (long)blockIdx.x * RPI + rr; r0 < L; r0 += BN_UR * step) {
            u16x8_t gv[BN_UR], xv8[BN_UR], mv[MODE == 1 ? BN_UR : 1], x2v8[X2 ? BN_UR : 1];
            unsigned mb[MODE == 3 ? BN_UR : 1];
#pragma unroll
            for (int u = 0; u < BN_UR; ++u) {      // every row's loads in flight together
                const long r = r0 + u * step;
                if (r < L) {
                    const long off = r * C + c;
                    gv[u] = *reinterpret_cast<const u16x8_t*>(g + off);
                    xv8[u] = *reinterpret_cast<const u16x8_t*>(x + off);
                    if constexpr (MODE == 1) mv[u] = *reinterpret_cast<const u16x8_t*>(msrc + off);
                    if constexpr (MODE == 3) mb[u] = reinterpret_cast<const uint8_t*>(msrc)[r * CG + cg];
                    if constexpr (X2) x2v8[u] = *reinterpret_cast<const u16x8_t*>(x2 + off);
                }
            }
#pragma unroll
            for (int u = 0; u < BN_UR; ++u) {
                if (r0 + u * step >= L) break;
                float gm[8], xv[8];
                unpack8(gv[u], gm);
                unpack8(xv8[u], xv);
                if constexpr (MODE == 1) {
                    float m[8];
                    unpack8(mv[u], m);
#pragma unroll
                    for (int j = 0; j < 8; ++j) gm[j] = m[j] > 0.f ? gm[j] : 0.f;
                } else if constexpr (MODE == 2) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) gm[j] = fmaf(xv[j], ms[j], mh[j]) > 0.f ? gm[j] : 0.f;
                } else if constexpr (MODE == 3) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) gm[j] = ((mb[u] >> j) & 1u) ? gm[j] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) { s[j] += gm[j]; q[j] += gm[j] * (xv[j] - mu[j]) * is[j]; }
                if constexpr (X2) {
                    float x2v[8];
                    unpack8(x2v8[u], x2v);
#pragma unroll
                    for (int j = 0; j < 8; ++j) q2[j] += gm[j] * (x2v[j] - mu2[j]) * is2[j];
                }
            }
        }
    }
    for (int pass = 0; pass < (X2 ? 2 : 1); ++pass) {
        float* out = pass ? slab2 : slab;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[0][t * 8 + j] = s[j];
            if constexpr (X2) red[1][t * 8 + j] = pass ? q2[j] : q[j];
            else red[1][t * 8 + j] = q[j];
        }
        __syncthreads();
        for (int cc = t; cc < C; cc += NT) {
            const int gg = cc >> 3, j = cc & 7;
            float a = 0.f, b = 0.f;
            for (int k = 0; k < RPI; ++k) { a += red[0][(k * CG + gg) * 8 + j]; b += red[1][(k * CG + gg) * 8 + j]; }
            out[(long)(2 * blockIdx.x) * C + cc] = a;
            out[(long)(2 * blockIdx.x + 1) * C + cc] = b;
        }
        __syncthreads();
    }
}

// sum partial rows -> dbeta (= sum gm), dgamma (= sum gm*xhat).  Optionally accumulate (+=).
__global__ void __launch_bounds__(NT) bn_bwd_finalize_kernel(const float* __restrict__ slab, int rows, int C,
                                                             float* dgamma, float* dbeta, int accumulate,
                                                             float* gacc, float* bacc) {
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), lr = threadIdx.x >> 6;
    __shared__ double red[2][4][64];
    double s = 0.0, q = 0.0;
    if (c < C)
        for (int r = lr; r < rows; r += 4) {
            s += slab[(long)(2 * r) * C + c];
            q += slab[(long)(2 * r + 1) * C + c];
        }
    red[0][lr][threadIdx.x & 63] = s;
    red[1][lr][threadIdx.x & 63] = q;
    __syncthreads();
    if (lr != 0 || c >= C) return;
    const int l = threadIdx.x;
    s = red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l];
    q = red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l];
    if (accumulate) { dbeta[c] += (float)s; dgamma[c] += (float)q; }
    else { dbeta[c] = (float)s; dgamma[c] = (float)q; }
    if (gacc) { gacc[c] += (float)q; bacc[c] += (float)s; }     // direct accumulation into param grads
}

// dx = gamma*invstd*(gm - dbeta/L - xhat*dgamma/L) = k*gm + x*A + B with per-channel k, A, B held in
// registers; optionally also a second BN's dx2 (shared gm) and/or gm itself.
// Specialised on the mask mode / second BN / outputs so unused coefficient arrays take no registers
// (occupancy).
template <int MODE, bool X2, bool DX, bool GMO>
__global__ void __launch_bounds__(NT) bn_bwd_apply_kernel(
    const bf16_t* __restrict__ g, const bf16_t* __restrict__ x, long L, int C,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ dgamma, const float* __restrict__ dbeta,
    const bf16_t* __restrict__ msrc, const float* __restrict__ mscale, const float* __restrict__ mshift,
    bf16_t* __restrict__ dx, const bf16_t* __restrict__ x2, const float* __restrict__ mean2,
    const float* __restrict__ invstd2, const float* __restrict__ gamma2, const float* __restrict__ dgamma2,
    const float* __restrict__ dbeta2, bf16_t* __restrict__ dx2, bf16_t* __restrict__ gm_out) {
    const int CG = C >> 3, RPI = NT / CG;
    const int t = threadIdx.x, cg = t % CG, rr = t / CG, c = cg * 8;
    if (rr >= RPI) return;
    const float invL = (float)(1.0 / (double)L);
    float k1[8], A1[8], B1[8];
    float k2[X2 ? 8 : 1], A2[X2 ? 8 : 1], B2[X2 ? 8 : 1], ms[MODE == 2 ? 8 : 1], mh[MODE == 2 ? 8 : 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float is = invstd[c + j], k = (gamma ? gamma[c + j] : 1.f) * is;
        const float dg = dgamma[c + j] * invL, db = dbeta[c + j] * invL;
        k1[j] = k; A1[j] = -k * is * dg; B1[j] = k * (mean[c + j] * is * dg - db);
        if constexpr (X2) {
            const float is2 = invstd2[c + j], kk = (gamma2 ? gamma2[c + j] : 1.f) * is2;
            const float dg2 = dgamma2[c + j] * invL, db2 = dbeta2[c + j] * invL;
            k2[j] = kk; A2[j] = -kk * is2 * dg2; B2[j] = kk * (mean2[c + j] * is2 * dg2 - db2);
        }
        if constexpr (MODE == 2) { ms[j] = mscale[c + j]; mh[j] = mshift[c + j]; }
    }
    // software-pipelined over rows like bn_apply_kernel: row r+step's loads are issued before row r's stores
    const long step = (long)gridDim.x * RPI;
    long r = (long)blockIdx.x * RPI + rr;
    if (r >= L) return;
    struct Ops {
        u16x8_t g, x, m, x2;
        unsigned mb;
    };
    auto load = [&](long row, Ops& o) {
        const long off = row * C + c;
        o.g = *reinterpret_cast<const u16x8_t*>(g + off);
        o.x = *reinterpret_cast<const u16x8_t*>(x + off);
        if constexpr (MODE == 1) o.m = *reinterpret_cast<const u16x8_t*>(msrc + off);
        if constexpr (MODE == 3) o.mb = reinterpret_cast<const uint8_t*>(msrc)[row * CG + cg];
        if constexpr (X2) o.x2 = *reinterpret_cast<const u16x8_t*>(x2 + off);
    };
    Ops cur, nxt;
    load(r, cur);
    for (; r < L; r += step) {
        load(r + step < L ? r + step : L - 1, nxt);
        const long off = r * C + c;
        float gm[8], xv[8], o[8];
        unpack8(cur.g, gm);
        unpack8(cur.x, xv);
        if constexpr (MODE == 1) {
            float m[8];
            unpack8(cur.m, m);
#pragma unroll
            for (int j = 0; j < 8; ++j) gm[j] = m[j] > 0.f ? gm[j] : 0.f;
        } else if constexpr (MODE == 2) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gm[j] = fmaf(xv[j], ms[j], mh[j]) > 0.f ? gm[j] : 0.f;
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j) gm[j] = ((cur.mb >> j) & 1u) ? gm[j] : 0.f;
        }
        if constexpr (DX) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = fmaf(k1[j], gm[j], fmaf(xv[j], A1[j], B1[j]));
            *reinterpret_cast<u16x8_t*>(dx + off) = pack8(o);
        }
        if constexpr (X2) {
            float x2v[8];
            unpack8(cur.x2, x2v);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = fmaf(k2[j], gm[j], fmaf(x2v[j], A2[j], B2[j]));
            *reinterpret_cast<u16x8_t*>(dx2 + off) = pack8(o);
        }
        if constexpr (GMO) *reinterpret_cast<u16x8_t*>(gm_out + off) = pack8(gm);
        cur = nxt;
    }
}

// BN apply / BN-backward apply: 512 blocks (2 per CU), each thread row walking many rows through the
// software pipeline; the generic 2048-block stream grid ran ResNet-50 2.7% slower, 1024 1.3% slower, 256 2% slower
// (profiles/resnet50_bn_grid_r4.txt, gpurun_out/r4_65-67)
inline unsigned bn_stream_grid(long work) {
    long g = (work + NT - 1) / NT;
    if (g > 512) g = 512;
    return (unsigned)(g < 1 ? 1 : g);
}

inline unsigned reduce_grid(long L, int C) {
    const int rpi = NT / (C / 8);
    long g = (L + rpi * BN_RMIN - 1) / (rpi * BN_RMIN);   // >= BN_RMIN rows per thread-row
    if (g > 512) g = 512;
    if (g < 1) g = 1;
    return (unsigned)g;
}
}  // namespace

PDNN_API int pdnn_bn_reduce_rows(long L, int C) { return (int)reduce_grid(L, C); }

// floats of `work` the finalize calls need for a slab of `rows` partial rows
PDNN_API int pdnn_bn_fin_work(int rows, int C) {
#if PDNN_BN_WIDE_FIN
    return 2 * (int)fin_rows(rows) * C;
#else
    return rows > 64 ? 2 * 64 * C : 0;
#endif
}

// work: >= pdnn_bn_fin_work(rows, C) floats of scratch for the level-1 reduction; cnt (optional): C/64 zeroed
// counters -> one launch (bn_slab_fused_kernel), left zeroed
PDNN_API int pdnn_bn_finalize(const float* slab, int rows, int C, double L, float eps, float momentum,
                              const float* gamma, const float* beta, float* run_mean, float* run_var,
                              float* mean_out, float* invstd_out, float* scale_out, float* shift_out,
                              float* work, unsigned* cnt, hipStream_t st) {
#if PDNN_BN_WIDE_FIN
    const FinFwd epi{L, eps, momentum, gamma, beta, run_mean, run_var, mean_out, invstd_out, scale_out, shift_out};
    const unsigned rb = fin_rows(rows);
    if (rb && cnt) {
        hipLaunchKernelGGL(bn_slab_fused_kernel<FinFwd>, dim3((C + 63) / 64, rb), dim3(NT), 0, st, slab, rows, C, work,
                           cnt, epi);
        PDNN_LAUNCH_RET;
    }
    if (rb) hipLaunchKernelGGL(bn_slab_level1_kernel, dim3((C + 63) / 64, rb), dim3(NT), 0, st, slab, rows, C, work);
    hipLaunchKernelGGL(bn_slab_final_kernel<FinFwd>, dim3((C + 63) / 64), dim3(NT), 0, st, rb ? work : slab,
                       rb ? (int)rb : rows, C, epi);
#else
    const float* src = slab;
    int r = rows;
    if (rows > 64) {
        hipLaunchKernelGGL(slab_reduce_kernel, dim3((C + 63) / 64, 64), dim3(NT), 0, st, slab, rows, C, work);
        src = work;
        r = 64;
    }
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(NT), 0, st, src, r, C, L, eps,
                       momentum, gamma, beta, run_mean, run_var, mean_out, invstd_out, scale_out, shift_out);
#endif
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_bn_eval_coeff(int C, float eps, const float* gamma, const float* beta, const float* rm,
                                const float* rv, float* scale, float* shift, hipStream_t st) {
    hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, eps, gamma, beta,
                       rm, rv, scale, shift);
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_bn_stats(const bf16_t* x, long L, int C, float* slab, hipStream_t st) {
    hipLaunchKernelGGL(bn_stats_kernel, dim3(reduce_grid(L, C)), dim3(NT), 0, st, x, L, C, slab);
    PDNN_LAUNCH_RET;
}

// mbits (optional, [L][C/8] bytes): sign bits of y for a mask-mode-3 backward
PDNN_API int pdnn_bn_apply(const bf16_t* x, long L, int C, const float* scale, const float* shift,
                           const bf16_t* res, const float* rscale, const float* rshift, int relu, bf16_t* y,
                           uint8_t* mbits, hipStream_t st) {
    const dim3 grid(bn_stream_grid(L * (C / 8)));
#define PDNN_BA(RES, RSC, RELU, MASK)                                                                  \
    hipLaunchKernelGGL((bn_apply_kernel<RES, RSC, RELU, MASK>), grid, dim3(NT), 0, st, x, L, C, scale, shift, res, \
                       rscale, rshift, y, mbits)
    if (mbits && relu) {
        if (res && rscale) PDNN_BA(true, true, true, true);
        else if (res) PDNN_BA(true, false, true, true);
        else PDNN_BA(false, false, true, true);
    } else if (res && rscale) { if (relu) PDNN_BA(true, true, true, false); else PDNN_BA(true, true, false, false); }
    else if (res) { if (relu) PDNN_BA(true, false, true, false); else PDNN_BA(true, false, false, false); }
    else { if (relu) PDNN_BA(false, false, true, false); else PDNN_BA(false, false, false, false); }
#undef PDNN_BA
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_bn_bwd_reduce(const bf16_t* g, const bf16_t* x, long L, int C, const float* mean,
                                const float* invstd, int mode, const bf16_t* msrc, const float* mscale,
                                const float* mshift, float* slab, const bf16_t* x2, const float* mean2,
                                const float* invstd2, float* slab2, hipStream_t st) {
#define PDNN_BWR(MODE, X2)                                                                                  \
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<MODE, X2>), dim3(reduce_grid(L, C)), dim3(NT), 0, st, g, x, L, C, \
                       mean, invstd, msrc, mscale, mshift, slab, x2, mean2, invstd2, slab2)
    const bool hx2 = x2 != nullptr;
    switch (mode) {
        case 1: if (hx2) PDNN_BWR(1, true); else PDNN_BWR(1, false); break;
        case 2: if (hx2) PDNN_BWR(2, true); else PDNN_BWR(2, false); break;
        case 3: if (hx2) PDNN_BWR(3, true); else PDNN_BWR(3, false); break;
        default: if (hx2) PDNN_BWR(0, true); else PDNN_BWR(0, false); break;
    }
#undef PDNN_BWR
    PDNN_LAUNCH_RET;
}

// dgamma/dbeta of this backward (consumed by bn_bwd_apply); gacc/bacc (optional): also added into the
// parameters' gradient accumulators.
PDNN_API int pdnn_bn_bwd_finalize(const float* slab, int rows, int C, float* dgamma, float* dbeta,
                                  int accumulate, float* work, float* gacc, float* bacc, unsigned* cnt,
                                  hipStream_t st) {
#if PDNN_BN_WIDE_FIN
    const FinBwd epi{dgamma, dbeta, accumulate, gacc, bacc};
    const unsigned rb = fin_rows(rows);
    if (rb && cnt) {
        hipLaunchKernelGGL(bn_slab_fused_kernel<FinBwd>, dim3((C + 63) / 64, rb), dim3(NT), 0, st, slab, rows, C, work,
                           cnt, epi);
        PDNN_LAUNCH_RET;
    }
    if (rb) hipLaunchKernelGGL(bn_slab_level1_kernel, dim3((C + 63) / 64, rb), dim3(NT), 0, st, slab, rows, C, work);
    hipLaunchKernelGGL(bn_slab_final_kernel<FinBwd>, dim3((C + 63) / 64), dim3(NT), 0, st, rb ? work : slab,
                       rb ? (int)rb : rows, C, epi);
#else
    const float* src = slab;
    int r = rows;
    if (rows > 64) {
        hipLaunchKernelGGL(slab_reduce_kernel, dim3((C + 63) / 64, 64), dim3(NT), 0, st, slab, rows, C, work);
        src = work;
        r = 64;
    }
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(NT), 0, st, src, r, C, dgamma,
                       dbeta, accumulate, gacc, bacc);
#endif
    PDNN_LAUNCH_RET;
}

PDNN_API int pdnn_bn_bwd_apply(const bf16_t* g, const bf16_t* x, long L, int C, const float* mean,
                               const float* invstd, const float* gamma, const float* dgamma,
                               const float* dbeta, int mode, const bf16_t* msrc, const float* mscale,
                               const float* mshift, bf16_t* dx, const bf16_t* x2, const float* mean2,
                               const float* invstd2, const float* gamma2, const float* dgamma2,
                               const float* dbeta2, bf16_t* dx2, bf16_t* gm_out, hipStream_t st) {
    const dim3 grid(bn_stream_grid(L * (C / 8)));
#define PDNN_BWA(MODE, X2, DX, GMO)                                                                              \
    hipLaunchKernelGGL((bn_bwd_apply_kernel<MODE, X2, DX, GMO>), grid, dim3(NT), 0, st, g, x, L, C, mean, invstd, \
                       gamma, dgamma, dbeta, msrc, mscale, mshift, dx, x2, mean2, invstd2, gamma2, dgamma2,      \
                       dbeta2, dx2, gm_out)
    const bool hx2 = x2 != nullptr, hdx = dx != nullptr, hgm = gm_out != nullptr;
    if (mode == 1) {
        if (hx2) { if (hgm) PDNN_BWA(1, true, true, true); else PDNN_BWA(1, true, true, false); }
        else if (hgm) { if (hdx) PDNN_BWA(1, false, true, true); else PDNN_BWA(1, false, false, true); }
        else PDNN_BWA(1, false, true, false);
    } else if (mode == 3) {
        if (hx2) { if (hgm) PDNN_BWA(3, true, true, true); else PDNN_BWA(3, true, true, false); }
        else if (hgm) { if (hdx) PDNN_BWA(3, false, true, true); else PDNN_BWA(3, false, false, true); }
        else PDNN_BWA(3, false, true, false);
    } else if (mode == 2) {
        if (hgm) PDNN_BWA(2, false, true, true); else PDNN_BWA(2, false, true, false);
    } else {
        if (hx2) PDNN_BWA(0, true, true, false); else PDNN_BWA(0, false, true, false);
    }
#undef PDNN_BWA
    PDNN_LAUNCH_RET;
}
