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
// Slab layout shared by every partial-statistics producer: STAT_BINS bins [64][2][C] fp32 (common.h) that the
// producers ADD their partial rows into (partial row i -> bin i % 64): slab[(2b)*C + c] += sum,
// slab[(2b+1)*C + c] += sum of squares (or, in backward, sum(g) / sum(g*xhat)).  The finalize reads the 64
// bins and leaves them zeroed for the next producer.
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
constexpr int BN_UR = PDNN_BN_UR, BN_RMIN = PDNN_BN_RMIN;

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

// Finalize of the STAT_BINS bins: block = one 64-channel column, 16 float4 channel groups x 16 bin lanes (4 bins
// each, all loads in flight together), fp64 sums; every element read is zeroed again by the thread that read it
// (the next producer adds into zeros; a bin buffer is reused only in stream order after this kernel).  Replaces a
// level-1 + last-arriver pass over one row pair per producer tile (up to 12544 rows: 7.7-20 us per call,
// gpurun_out/r5_01).
template <class Epi>
__global__ void __launch_bounds__(NT) bn_bins_final_kernel(float* __restrict__ bins, int C, Epi epi) {
    const int col = blockIdx.x, ch = threadIdx.x & 15, lane = threadIdx.x >> 4;
    const int c0 = col * 64 + ch * 4;
    constexpr int PER = STAT_BINS / 16;
    double sd[4] = {0, 0, 0, 0}, qd[4] = {0, 0, 0, 0};
    if (c0 < C) {
        float4 a[PER], b[PER];
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int r = lane + 16 * j;
            a[j] = *reinterpret_cast<const float4*>(bins + (long)(2 * r) * C + c0);
            b[j] = *reinterpret_cast<const float4*>(bins + (long)(2 * r + 1) * C + c0);
        }
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const int r = lane + 16 * j;
            sd[0] += a[j].x; sd[1] += a[j].y; sd[2] += a[j].z; sd[3] += a[j].w;
            qd[0] += b[j].x; qd[1] += b[j].y; qd[2] += b[j].z; qd[3] += b[j].w;
            *reinterpret_cast<float4*>(bins + (long)(2 * r) * C + c0) = z;
            *reinterpret_cast<float4*>(bins + (long)(2 * r + 1) * C + c0) = z;
        }
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
        float* row = stat_row(slab, blockIdx.x, C);
        stat_add(row + c, a);
        stat_add(row + C + c, b);
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
            float* row = stat_row(out, blockIdx.x, C);
            stat_add(row + cc, a);
            stat_add(row + C + cc, b);
        }
        __syncthreads();
    }
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

// slab = STAT_BINS bins [64][2][C] (common.h), left zeroed.  rows: kept in the signature (= STAT_BINS)
PDNN_API int pdnn_bn_finalize(float* slab, int rows, int C, double L, float eps, float momentum,
                              const float* gamma, const float* beta, float* run_mean, float* run_var,
                              float* mean_out, float* invstd_out, float* scale_out, float* shift_out, hipStream_t st) {
    if (rows != STAT_BINS) return (int)hipErrorInvalidValue;
    const FinFwd epi{L, eps, momentum, gamma, beta, run_mean, run_var, mean_out, invstd_out, scale_out, shift_out};
    hipLaunchKernelGGL(bn_bins_final_kernel<FinFwd>, dim3((C + 63) / 64), dim3(NT), 0, st, slab, C, epi);
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
// parameters' gradient accumulators.  slab = STAT_BINS bins, left zeroed.
PDNN_API int pdnn_bn_bwd_finalize(float* slab, int rows, int C, float* dgamma, float* dbeta, int accumulate,
                                  float* gacc, float* bacc, hipStream_t st) {
    if (rows != STAT_BINS) return (int)hipErrorInvalidValue;
    const FinBwd epi{dgamma, dbeta, accumulate, gacc, bacc};
    hipLaunchKernelGGL(bn_bins_final_kernel<FinBwd>, dim3((C + 63) / 64), dim3(NT), 0, st, slab, C, epi);
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
