// Shared pieces of the direct (non-implicit-GEMM) convolution kernels: conv3x3.hip (LDS-halo 3x3, pixel
// panel and A-stationary 1x1) and stem.hip (7x7 / stride-2 stem).  Argument block, operand masking, the
// LDS halo swizzle, the BatchNorm-backward operand prologue and the common epilogue (plain / residual /
// BN statistics / fused BN backward) -- one slab row pair per (pixel tile, wave), 64 pixels each.
#pragma once
#include "gemm_common.h"
#include "tuning.h"

namespace {
using namespace pg;

constexpr int C3_BM = 256;
enum { C3_PLAIN = 0, C3_STATS = 1, C3_BNB = 2, C3_RES = 3 };

struct C3Args {
    const bf16_t* x;     // [P][C]  NHWC input
    const bf16_t* w;     // [N][3][3][C]
    bf16_t* y;           // [P][N]
    int Nimg, H, W, C, N, P;
    FastDiv dW, dH;
    int tiles, ntiles;
    int halo_max;        // pixels of the largest halo (LDS layout)
    float* stats;
    const bf16_t* res;
    const uint8_t* rmask;  // C3_RES: residual masked by these ReLU bits ([P][N/8] bytes), or null
    const bf16_t* ep_x;
    const float *ep_mean, *ep_invstd, *ep_mscale, *ep_mshift;
    // PRE operand prologue (BatchNorm backward apply of the layer whose gradient is the input): the staged
    // operand is dt = k*gm + A*t + B per channel (pdnn_bn_bwd_apply's formula, same rounding) with gm = x;
    // the own pixels' dt is also written to pre_out (the weight gradient's operand)
    const bf16_t* pre_t;
    const float *pre_mean, *pre_invstd, *pre_gamma, *pre_dgamma, *pre_dbeta;
    bf16_t* pre_out;
    // fp8 halo kernel (conv3x3.hip F8 != 0): w is e4m3 bytes; the staged operand is quantised with f8_scale[0]
    // (delayed scaling), its |max| goes to the FP8_AMAX_PARTS partials f8_amax, acc is dequantised by
    // f8_inv[0] * f8_winv[0]
    const float *f8_scale, *f8_inv, *f8_winv;
    float* f8_amax;
    // forward operand prologue (conv3x3.hip FP): the staged operand is relu(x * pro_sc[c] + pro_sh[c]) -- the BN + ReLU
    // of the layer that produced x, so its output never has to be materialised (bn_apply's formula and rounding)
    const float *pro_sc, *pro_sh;
};

// per-channel coefficients of 8 consecutive channels c .. c+7 (batchnorm.hip bn_bwd_apply_kernel)
struct PreCoef {
    float k[8], A[8], B[8];
};
__device__ __forceinline__ void pre_coef(const C3Args& a, int c, PreCoef& pc) {
    const float invL = (float)(1.0 / (double)a.P);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float is = a.pre_invstd[c + j], k = (a.pre_gamma ? a.pre_gamma[c + j] : 1.f) * is;
        const float dg = a.pre_dgamma[c + j] * invL, db = a.pre_dbeta[c + j] * invL;
        pc.k[j] = k;
        pc.A[j] = -k * is * dg;
        pc.B[j] = k * (a.pre_mean[c + j] * is * dg - db);
    }
}
__device__ __forceinline__ u16x8_t pre_apply(const PreCoef& pc, const u16x8_t& gv, const u16x8_t& tv) {
    float gm[8], t[8], o[8];
    unpack8(gv, gm);
    unpack8(tv, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(pc.k[j], gm[j], fmaf(t[j], pc.A[j], pc.B[j]));
    return pack8(o);
}

// The same apply with the coefficients of the chunk's CH channels in LDS (coef: [3][CH] = k, A, B), c = channel
// index in the chunk: keeps 24 VGPRs per 8 channels free for more operand loads in flight (halo staging)
template <int CH>
__device__ __forceinline__ void pre_coef_lds(const C3Args& a, int c0, float* coef, int tid) {
    const float invL = (float)(1.0 / (double)a.P);
    for (int c = tid; c < CH; c += 256) {
        const float is = a.pre_invstd[c0 + c], k = (a.pre_gamma ? a.pre_gamma[c0 + c] : 1.f) * is;
        const float dg = a.pre_dgamma[c0 + c] * invL, db = a.pre_dbeta[c0 + c] * invL;
        coef[c] = k;
        coef[CH + c] = -k * is * dg;
        coef[2 * CH + c] = k * (a.pre_mean[c0 + c] * is * dg - db);
    }
}
template <int CH>
__device__ __forceinline__ u16x8_t pre_apply_lds(const float* coef, int c, const u16x8_t& gv, const u16x8_t& tv) {
    float gm[8], t[8], o[8], k[8], A[8], B[8];
    unpack8(gv, gm);
    unpack8(tv, t);
    *reinterpret_cast<float4*>(k) = *reinterpret_cast<const float4*>(coef + c);
    *reinterpret_cast<float4*>(k + 4) = *reinterpret_cast<const float4*>(coef + c + 4);
    *reinterpret_cast<float4*>(A) = *reinterpret_cast<const float4*>(coef + CH + c);
    *reinterpret_cast<float4*>(A + 4) = *reinterpret_cast<const float4*>(coef + CH + c + 4);
    *reinterpret_cast<float4*>(B) = *reinterpret_cast<const float4*>(coef + 2 * CH + c);
    *reinterpret_cast<float4*>(B + 4) = *reinterpret_cast<const float4*>(coef + 2 * CH + c + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = fmaf(k[j], gm[j], fmaf(t[j], A[j], B[j]));
    return pack8(o);
}

// forward prologue coefficients of the chunk's CH channels in LDS (coef: [2][CH] = scale, shift) and its apply
template <int CH>
__device__ __forceinline__ void fpro_coef_lds(const C3Args& a, int c0, float* coef, int tid) {
    for (int c = tid; c < CH; c += 256) {
        coef[c] = a.pro_sc[c0 + c];
        coef[CH + c] = a.pro_sh[c0 + c];
    }
}
template <int CH>
__device__ __forceinline__ u16x8_t fpro_apply_lds(const float* coef, int c, const u16x8_t& v) {
    float x[8], sc[8], sh[8];
    unpack8(v, x);
    *reinterpret_cast<float4*>(sc) = *reinterpret_cast<const float4*>(coef + c);
    *reinterpret_cast<float4*>(sc + 4) = *reinterpret_cast<const float4*>(coef + c + 4);
    *reinterpret_cast<float4*>(sh) = *reinterpret_cast<const float4*>(coef + CH + c);
    *reinterpret_cast<float4*>(sh + 4) = *reinterpret_cast<const float4*>(coef + CH + c + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = fmaxf(fmaf(x[j], sc[j], sh[j]), 0.f);
    return pack8(x);
}

// v if ok else 0, as four 32-bit ANDs (a u16x8 AND with a 16-bit mask vector lowers to per-half sdwa/perm ops)
__device__ __forceinline__ u16x8_t mask16(const u16x8_t& v, bool ok) {
    const uint32_t m = ok ? 0xFFFFFFFFu : 0u;
    uint4 u = __builtin_bit_cast(uint4, v);
    u.x &= m; u.y &= m; u.z &= m; u.w &= m;
    return __builtin_bit_cast(u16x8_t, u);
}

__device__ __forceinline__ u16x8_t c3_zero8() {
    u16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
    return z;
}

// halo image: pixel hp = 128 bytes (64 channels), 16-byte chunk q stored at q ^ ((hp >> 1) & 7)
__device__ __forceinline__ int halo_off(int hp, int q) {   // bf16 elements
    return hp * 64 + ((q ^ ((hp >> 1) & 7)) << 3);
}

// ---------------- epilogue: lane holds y[pixel m = wave*64 + fm*16 + (lane&15)][n = fn*16 + 4*(lane>>4) + j]
// Processed one fragment pair (fn, fn+1) at a time.  The operands a pair reads (residual or BN input t, the
// residual mask words) are loaded one pair AHEAD, before the current
// pair's stores, and unconditionally (rows past P read row 0 and are never stored): s_waitcnt vmcnt counts
// stores too on gfx9, so loads issued after a pair's stores waited for them and serialised one store drain +
// load latency per pair (the GPT-2 GEMM epilogues lost 13-20 us per call that way, gpurun_out/r4_13-14).
template <int NB, int EPI>
struct C3PairOps {
    static constexpr bool RES = EPI == C3_RES, BNB = EPI == C3_BNB;
    u16x4_t tv[(RES || BNB) ? 2 : 1][4];
    uint32_t mw[RES ? 4 : 1];
};

template <int NB, int EPI>
__device__ __forceinline__ void c3_load_pair(const C3Args& a, const long (&lrow)[4], int n0, int lg, int fp,
                                             C3PairOps<NB, EPI>& o) {
    constexpr bool RES = EPI == C3_RES, BNB = EPI == C3_BNB;
    if constexpr (RES) {
        // mask bits of this pair's 32 channels: ONE aligned 32-bit load per pixel (bit c = channel n0 + 32*fp + c),
        // not a byte load per fragment (that doubled the epilogue's memory instructions: ResNet-50 stage-1 conv1
        // data gradient 239 -> 341 us with the mask, gpurun_out/r3_18)
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
            o.mw[fm] = a.rmask ? *reinterpret_cast<const uint32_t*>(a.rmask + ((lrow[fm] + n0 + 32 * fp) >> 3))
                               : 0xFFFFFFFFu;
    }
    if constexpr (RES || BNB) {
        const bf16_t* src = BNB ? a.ep_x : a.res;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int n = n0 + (2 * fp + h) * 16 + 4 * lg;
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) o.tv[h][fm] = *reinterpret_cast<const u16x4_t*>(src + lrow[fm] + n);
        }
    }
}

// orow[fm]: element offset of this lane's output row in y (and in the epilogue operands laid out like y)
template <int NB, int EPI>
__device__ __forceinline__ void c3_epilogue_rows(const C3Args& a, f32x4_t (&acc)[4][NB / 16], int tile,
                                                 const long (&orow)[4], int n0, int wave, int lane,
                                                 const bool (&pv)[4]) {
    constexpr int FN = NB / 16, NP = FN / 2;
    constexpr bool RES = EPI == C3_RES;
    const int lg = lane >> 4;
    long lrow[4];
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) lrow[fm] = pv[fm] ? orow[fm] : 0;
    C3PairOps<NB, EPI> cur, nxt;
    if constexpr (NP > 1) c3_load_pair<NB, EPI>(a, lrow, n0, lg, 0, cur);
    else if constexpr (RES) {
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
            cur.mw[fm] = a.rmask ? *reinterpret_cast<const uint32_t*>(a.rmask + ((lrow[fm] + n0) >> 3)) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int fp = 0; fp < NP; ++fp) {
        if (fp + 1 < NP) c3_load_pair<NB, EPI>(a, lrow, n0, lg, fp + 1, nxt);
        uint32_t pk[4][2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int fn = 2 * fp + h;
            const int n = n0 + fn * 16 + 4 * lg;
            // fused BN backward: q accumulates sum gm * t; sum gm * xhat = invstd * (sum gm t - mean * sum gm) is
            // formed at the flush, so mean / invstd are not live through the fragment loop
            float s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
            float bms[4], bmh[4];
            if constexpr (NP == 1 && (RES || EPI == C3_BNB)) {
                // one pair (the 4 x 32 A-stationary kernels, at the register limit): only this half's operand live
                const bf16_t* src = EPI == C3_BNB ? a.ep_x : a.res;
#pragma unroll
                for (int fm = 0; fm < 4; ++fm)
                    cur.tv[h][fm] = pv[fm] ? *reinterpret_cast<const u16x4_t*>(src + orow[fm] + n) : u16x4_t{0, 0, 0, 0};
            }
            if constexpr (EPI == C3_BNB) {     // (per-channel tables: L2-resident, not prefetched -- registers)
                const float4 m4 = *reinterpret_cast<const float4*>(a.ep_mscale + n);
                const float4 h4 = *reinterpret_cast<const float4*>(a.ep_mshift + n);
                bms[0] = m4.x; bms[1] = m4.y; bms[2] = m4.z; bms[3] = m4.w;
                bmh[0] = h4.x; bmh[1] = h4.y; bmh[2] = h4.z; bmh[3] = h4.w;
            }
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
                const bool ok = pv[fm];
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = acc[fm][fn][j];
                if constexpr (RES) {
                    const uint32_t mb = cur.mw[fm] >> (16 * h + 4 * lg);
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] += ((mb >> j) & 1) ? bf2f(cur.tv[h][fm][j]) : 0.f;
                }
                if constexpr (EPI == C3_BNB) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float tt = bf2f(cur.tv[h][fm][j]);
                        const float gm = (ok && fmaf(tt, bms[j], bmh[j]) > 0.f) ? bf2f(f2bf(v[j])) : 0.f;
                        v[j] = gm;
                        s[j] += gm;
                        q[j] += gm * tt;
                    }
                } else if constexpr (EPI == C3_STATS) {
                    if (ok) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float r = bf2f(f2bf(v[j]));
                            s[j] += r;
                            q[j] += r * r;
                        }
                    }
                }
                pk[fm][h][0] = pk2bf(v[0], v[1]);
                pk[fm][h][1] = pk2bf(v[2], v[3]);
            }
            if constexpr (EPI == C3_STATS || EPI == C3_BNB) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    s[j] = row16_sum(s[j]);
                    q[j] = row16_sum(q[j]);
                }
                {
                    float* ps = stat_row(a.stats, (long)tile * 4 + wave, a.N) + n;
                    if constexpr (EPI == C3_BNB) {
                        // lane lm in 4..7 adds column j = lm - 4's sum gm * xhat: only its own mean / invstd
                        const int j = lane & 3;
                        if ((lane & 12) == 4) {
                            const float qj = (sel4(q, j) - a.ep_mean[n + j] * sel4(s, j)) * a.ep_invstd[n + j];
                            q[0] = q[1] = q[2] = q[3] = qj;
                        }
                    }
                    stat_add_frag(ps, ps + a.N, lane, s, q, true);
                }
            }
        }
        // permlane16_swap pairs the two fragments: every lane then holds 8 consecutive channels (16 bytes)
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const auto s0 = __builtin_amdgcn_permlane16_swap(pk[fm][0][0], pk[fm][1][0], false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(pk[fm][0][1], pk[fm][1][1], false, false);
            const int n = n0 + (2 * fp + (lg & 1)) * 16 + 8 * (lg >> 1);
            if (pv[fm]) *reinterpret_cast<uint4*>(a.y + orow[fm] + n) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
        }
        if (fp + 1 < NP) cur = nxt;
    }
}

// output rows = the tile's pixels in order (row length a.N)
template <int NB, int EPI>
__device__ __forceinline__ void c3_epilogue(const C3Args& a, f32x4_t (&acc)[4][NB / 16], int tile, int p0, int n0,
                                            int wave, int lane, const bool (&pv)[4]) {
    long orow[4];
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) orow[fm] = (long)(p0 + wave * 64 + fm * 16 + (lane & 15)) * a.N;
    c3_epilogue_rows<NB, EPI>(a, acc, tile, orow, n0, wave, lane, pv);
}

}  // namespace
