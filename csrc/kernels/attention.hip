// Fused causal attention for head dim 64 (GPT-2; SURVEY.md §2.8 K-18 "flash-style attention"), bf16
// operands, fp32 softmax/accumulation, on the gfx950 MFMA 16x16x32 bf16 instruction.
//
// Layout: q, k, v are column blocks of the packed c_attn output qkv[B*T][3D] (ld = 3D): head h of
// token t of sequence b lives at row b*T + t, columns h*64 (q), D + h*64 (k), 2D + h*64 (v).  The output
// o[B*T][D] and the gradient dqkv[B*T][3D] use the same packing, so no head split/merge copies exist.
//
// Forward (one block = 128 queries of one (b, h), 4 waves x 32 queries; K/V tiles of 64 keys
// register-staged into double-buffered LDS, one barrier per tile):
//   S^T = K Q^T  ->  lane holds S^T[key = 16f + 4g + r][query = lane & 15]  (g = lane >> 4)
//   online softmax per query (= per lane; the 4 lane groups are combined by two xor-shuffles)
//   O^T += V^T P^T: P^T is consumed straight from the accumulator registers as the B operand of the
//   next MFMA (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"); the k order
//   inside an MFMA step is permuted (element e of lane group g = key 4g + e or 16 + 4g + e - 4), and the
//   V^T operand is read with ds_read_b64_tr_b16 from exactly those permuted key rows, so no LDS round trip
//   of P is needed.
// Saves lse2 = m + log2(sum) (base-2, scaled-score domain) per query for the backward.
//
// Backward (FlashAttention-2 split, both kernels recompute P from lse2):
//   attn_bwd_dkdv: one block = 64 keys (4 waves x 16 keys), loop over query tiles q >= key:
//       S = Q K^T, P, dV^T += dO^T P, dP = dO V^T, dS = P (dP - delta), dK^T += Q^T dS
//   attn_bwd_dq:   one block = 64 queries (4 waves x 16 queries), loop over key tiles k <= query:
//       S^T = K Q^T, P^T, dP^T = V dO^T, dS^T, dQ^T += K^T dS^T
//   delta[q] = sum_d dO[q][d] O[q][d] comes from attn_bwd_delta.
#include "common.h"
#include "tuning.h"

// Block order over (query or key tile, head, sequence): 0 = 3-D grid, heavy tiles first inside each (head, sequence);
// 1 = 1-D grid, heavy tiles first over the WHOLE grid (the dispatcher hands out blocks in index order, so the last
// blocks to start are the lightest ones and the causal triangle's tail is short)
#ifndef PDNN_ATTN_ORDER
#define PDNN_ATTN_ORDER 1
#endif

namespace {
constexpr int HD = 64;          // head dim

// (tile, head, sequence) of this block; heavy = tile index giving the most work first
__device__ __forceinline__ void attn_block(int ntile, int H, bool heavy_is_last, int& tile, int& h, int& b) {
#if PDNN_ATTN_ORDER == 1
    const int t = blockIdx.x, HB = gridDim.x / ntile;      // 1-D grid of ntile x H x B blocks
    const int r = t / HB, hb = t - r * HB;
    tile = heavy_is_last ? ntile - 1 - r : r;
    h = hb % H;
    b = hb / H;
#else
    tile = heavy_is_last ? ntile - 1 - (int)blockIdx.x : (int)blockIdx.x;
    h = blockIdx.y;
    b = blockIdx.z;
#endif
}
constexpr int NTA = 256;
constexpr float RESC = 8.f;     // forward lazy-rescale threshold (log2 units)
constexpr float LOG2E = 1.4426950408889634f;

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// [64][64] bf16 tile image, 128-byte rows, 16-byte chunk c of row r at chunk c ^ ((r >> 1) & 7)
__device__ __forceinline__ int toff(int row, int chunk) { return row * HD + ((chunk ^ ((row >> 1) & 7)) << 3); }

// K-major fragment: lane -> row (row0 + (lane & 15)), k = 32 ks + 8 (lane >> 4) .. +7
__device__ __forceinline__ bf16x8_t frag_rows(const bf16_t* img, int row0, int ks, int lane) {
    const int row = row0 + (lane & 15);
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(img + toff(row, ks * 4 + (lane >> 4))));
}

// Transposed fragment for an MFMA step over 32 tile rows [32 kk, 32 kk + 32) in the permuted order of
// an accumulator-sourced operand: lane (col = col0 + (lane & 15), group g) receives rows
// 32kk + 4g + 0..3 (elements 0-3) and 32kk + 16 + 4g + 0..3 (elements 4-7) of column col.
__device__ __forceinline__ bf16x8_t frag_tr_perm(const bf16_t* img, int col0, int kk, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = col0 + 4 * p;
    const int r0 = 32 * kk + 4 * g + q;
    const bf16_t* p0 = img + toff(r0, col >> 3) + (col & 7);
    const bf16_t* p1 = img + toff(r0 + 16, col >> 3) + (col & 7);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
}

// two fp32 accumulator fragments (rows 4g + r of fragment a and b) -> one bf16 B operand (permuted k)
__device__ __forceinline__ bf16x8_t pack_acc(const f32x4_t& a, const f32x4_t& b) {
    s16x8 v;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[r] = (short)f2bf(a[r]);
        v[4 + r] = (short)f2bf(b[r]);
    }
    return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ f32x4_t mfma(const bf16x8_t& a, const bf16x8_t& b, const f32x4_t& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// global fragment load: row-major [rows][ld] source, lane -> row (lane & 15), 8 k at 32 ks + 8 g
__device__ __forceinline__ bf16x8_t gfrag(const bf16_t* base, long ld, int ks, int lane) {
    const bf16_t* p = base + (long)(lane & 15) * ld + ks * 32 + 8 * (lane >> 4);
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(p));
}

// 64 x 64 tile: 256 threads x 2 chunks
struct TileLd {
    u16x8_t r[2];
    __device__ __forceinline__ void load(const bf16_t* src, long ld, int tid) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = (tid >> 3) + 32 * i, ch = tid & 7;
            r[i] = *reinterpret_cast<const u16x8_t*>(src + (long)row * ld + ch * 8);
        }
    }
    __device__ __forceinline__ void store(bf16_t* img, int tid) const {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int row = (tid >> 3) + 32 * i, ch = tid & 7;
            *reinterpret_cast<u16x8_t*>(img + toff(row, ch)) = r[i];
        }
    }
};

// max / sum over the four 16-lane rows (lanes l, l^16, l^32, l^48) by VALU lane swaps: v_permlane16_swap /
// v_permlane32_swap with both operands v return (v, partner) in some order per lane, so combining the pair is
// the xor-16 / xor-32 step (no ds_bpermute round trip through the LDS pipe)
__device__ __forceinline__ float pl16(float v, bool mx) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float a = __uint_as_float(r[0]), b = __uint_as_float(r[1]);
    return mx ? fmaxf(a, b) : a + b;
}
__device__ __forceinline__ float pl32(float v, bool mx) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float a = __uint_as_float(r[0]), b = __uint_as_float(r[1]);
    return mx ? fmaxf(a, b) : a + b;
}
__device__ __forceinline__ float rmax4(float v) { return pl32(pl16(v, true), true); }
__device__ __forceinline__ float rsum4(float v) { return pl32(pl16(v, false), false); }

// ---------------------------------------------------------------------------------------------- forward
__global__ void __launch_bounds__(NTA) attn_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                       float* __restrict__ lse2, int T, int H, float scale, int causal) {
    __shared__ __attribute__((aligned(16))) bf16_t smem[2][2][64 * HD];     // [buf][K|V]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const int nqb = T / 128;
    int qb, h, b;
    attn_block(nqb, H, true, qb, h, b);              // heavy (late) query tiles first
    const int D = H * HD;
    const long ld = 3L * D;
    const bf16_t* Q = qkv + (long)b * T * ld + h * HD;
    const bf16_t* Kp = Q + D;
    const bf16_t* Vp = Q + 2 * D;
    const int q0 = qb * 128 + 32 * w;                // this wave's 32 queries
    const float c = scale * LOG2E;

    bf16x8_t qf[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[f][ks] = gfrag(Q + (long)(q0 + 16 * f) * ld, ld, ks, lane);

    f32x4_t o[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) o[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

    const int nkb = causal ? (qb * 128 + 128) / 64 : T / 64;
    // K/V tiles: prefetch distance 2 (two register stages + two LDS buffers).  The per-tile compute of a
    // d=64 head is short, so with distance 1 every iteration waited out most of a global-load round trip
    // (causal and full attention took the same time: latency-, not throughput-bound).
    TileLd ka, va, kn, vn;
    ka.load(Kp, ld, tid);
    va.load(Vp, ld, tid);
    ka.store(smem[0][0], tid);
    va.store(smem[0][1], tid);
    if (nkb > 1) {
        kn.load(Kp + 64L * ld, ld, tid);
        vn.load(Vp + 64L * ld, ld, tid);
    }
    __syncthreads();
    // tile kb is in LDS buffer kb & 1; (hk, hv) hold tile kb + 1 in flight; (fk, fv) are free for kb + 2
    auto step = [&](const int kb, TileLd& hk, TileLd& hv, TileLd& fk, TileLd& fv) {
        const int cur = kb & 1;
        if (kb + 2 < nkb) {
            fk.load(Kp + (long)(kb + 2) * 64 * ld, ld, tid);
            fv.load(Vp + (long)(kb + 2) * 64 * ld, ld, tid);
        }
        const int k0 = kb * 64;
        if (!causal || k0 <= q0 + 31) {              // wave-uniform: tile not entirely above the diagonal
            const bf16_t* Ki = smem[cur][0];
            const bf16_t* Vi = smem[cur][1];
            f32x4_t s[4][2];
#pragma unroll
            for (int kf = 0; kf < 4; ++kf) {
                const bf16x8_t a0 = frag_rows(Ki, 16 * kf, 0, lane), a1 = frag_rows(Ki, 16 * kf, 1, lane);
#pragma unroll
                for (int f = 0; f < 2; ++f) {
                    f32x4_t z = {0.f, 0.f, 0.f, 0.f};
                    z = mfma(a0, qf[f][0], z);
                    s[kf][f] = mfma(a1, qf[f][1], z);
                }
            }
            // VALU budget per tile is what bounds a d=64 head (32 MFMAs vs ~32 softmax elements per lane):
            // the causal mask runs only on diagonal tiles (wave-uniform branch), the softmax scale is folded
            // into the exponent's FMA, exp2 is the raw v_exp_f32 (arguments <= 0; underflow to 0 is
            // exactly what softmax wants), and O is rescaled only when some row maximum moved.
            const bool diag = causal && k0 + 63 > q0;
            if (diag) {
#pragma unroll
                for (int f = 0; f < 2; ++f) {
                    const int qi = q0 + 16 * f + (lane & 15);
#pragma unroll
                    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (k0 + 16 * kf + 4 * g + r > qi) s[kf][f][r] = -INFINITY;
                }
            }
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                float mx = -INFINITY;
#pragma unroll
                for (int kf = 0; kf < 4; ++kf)
#pragma unroll
                    for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[kf][f][r]);
                // lazy rescale (cdna_hip_programming.md T13): the running maximum moves only when some query's tile
                // maximum exceeds it by more than 2^RESC in probability terms; below that the tile's P values use
                // the stale maximum (P <= 2^RESC, exact after the final 1 / l) and O and l keep their scale
                const float mt = rmax4(mx) * c;                     // scaled-score domain (c > 0)
                const bool moved = __any(mt > m[f] + RESC);
                const float mn = moved ? fmaxf(m[f], mt) : m[f];
                const float alpha = moved ? __builtin_amdgcn_exp2f(m[f] - mn) : 1.f;
                float rs = 0.f;
#pragma unroll
                for (int kf = 0; kf < 4; ++kf)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float p = __builtin_amdgcn_exp2f(fmaf(s[kf][f][r], c, -mn));
                        s[kf][f][r] = p;
                        rs += p;
                    }
                l[f] = l[f] * alpha + rs;                           // this lane's partial; rows summed at the end
                m[f] = mn;
                if (moved) {
#pragma unroll
                    for (int df = 0; df < 4; ++df) o[df][f] *= alpha;
                }
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16x8_t pb[2];
#pragma unroll
                for (int f = 0; f < 2; ++f) pb[f] = pack_acc(s[2 * kk][f], s[2 * kk + 1][f]);
#pragma unroll
                for (int df = 0; df < 4; ++df) {
                    const bf16x8_t vfr = frag_tr_perm(Vi, 16 * df, kk, lane);
#pragma unroll
                    for (int f = 0; f < 2; ++f) o[df][f] = mfma(vfr, pb[f], o[df][f]);
                }
            }
        }
        if (kb + 1 < nkb) {
            hk.store(smem[cur ^ 1][0], tid);
            hv.store(smem[cur ^ 1][1], tid);
        }
        __syncthreads();
    };
    for (int kb = 0; kb < nkb; kb += 2) {            // unrolled by 2: register stages are compile-time
        step(kb, kn, vn, ka, va);
        if (kb + 1 < nkb) step(kb + 1, ka, va, kn, vn);
    }
    // lane holds O^T[d = 16 df + 4 g + r][q = q0 + 16 f + (lane & 15)]
#pragma unroll
    for (int f = 0; f < 2; ++f) {
        const int qi = q0 + 16 * f + (lane & 15);
        l[f] = rsum4(l[f]);
        const float inv = 1.f / l[f];
        bf16_t* op = out + ((long)b * T + qi) * D + h * HD;
#pragma unroll
        for (int df = 0; df < 4; ++df) {
            u16x4_t v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = f2bf(o[df][f][r] * inv);
            *reinterpret_cast<u16x4_t*>(op + 16 * df + 4 * g) = v;
        }
        if (g == 0) lse2[((long)b * H + h) * T + qi] = m[f] + __log2f(l[f]);
    }
}

// ---------------------------------------------------------------------------------------------- backward
// delta[b][h][t] = sum_d dO . O   (one thread per (row, head), 8 x 16-byte loads each)
__global__ void __launch_bounds__(NTA) attn_bwd_delta_kernel(const bf16_t* __restrict__ o, const bf16_t* __restrict__ dO,
                                                             float* __restrict__ delta, int BT, int T, int H) {
    const long i = (long)blockIdx.x * NTA + threadIdx.x;
    if (i >= (long)BT * H) return;
    const long row = i / H;
    const int h = (int)(i - row * H);
    const int D = H * HD;
    const bf16_t* a = o + row * D + h * HD;
    const bf16_t* bb = dO + row * D + h * HD;
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float x[8], y[8];
        unpack8(*reinterpret_cast<const u16x8_t*>(a + 8 * c), x);
        unpack8(*reinterpret_cast<const u16x8_t*>(bb + 8 * c), y);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += x[j] * y[j];
    }
    const long bidx = row / T, t = row - bidx * T;
    delta[(bidx * H + h) * T + t] = s;
}

// dK, dV for 64 NF keys per block (wave w: NF 16-key fragments from k0 = 64 NF kb + 16 NF w); loop over 64-query
// tiles.  NF = 2 reads every Q / dO fragment out of LDS once for two key fragments (see attn_bwd_dq_kernel).
template <int NF>
__global__ void __launch_bounds__(NTA) attn_bwd_dkdv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dO,
                                                            const float* __restrict__ lse2, const float* __restrict__ delta,
                                                            bf16_t* __restrict__ dqkv, int T, int H, float scale,
                                                            int causal) {
    __shared__ __attribute__((aligned(16))) bf16_t smem[2][2][64 * HD];     // [buf][Q|dO]
    // the query tile's lse2 / delta ride along with its Q / dO tile through LDS: loaded from global memory in the
    // compute loop they were waited on behind the next tile's prefetch loads (vmcnt is in order), every tile
    __shared__ __attribute__((aligned(16))) float lsd[2][2][64];              // [buf][lse2|delta][query]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const int nkb = T / (64 * NF);
    int kb, h, b;
    attn_block(nkb, H, false, kb, h, b);             // early key tiles have the most work: launched first
    const int D = H * HD;
    const long ld = 3L * D;
    const bf16_t* Q = qkv + (long)b * T * ld + h * HD;
    const bf16_t* Kp = Q + D;
    const bf16_t* Vp = Q + 2 * D;
    const bf16_t* dOp = dO + (long)b * T * D + h * HD;
    const float* L2 = lse2 + ((long)b * H + h) * T;
    const float* Dl = delta + ((long)b * H + h) * T;
    const int k0 = kb * 64 * NF + 16 * NF * w;
    const float c = scale * LOG2E;

    bf16x8_t kf[NF][2], vf[NF][2];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            kf[f][ks] = gfrag(Kp + (long)(k0 + 16 * f) * ld, ld, ks, lane);
            vf[f][ks] = gfrag(Vp + (long)(k0 + 16 * f) * ld, ld, ks, lane);
        }
    f32x4_t dv[NF][4], dk[NF][4];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) dv[f][i] = dk[f][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int qb0 = causal ? kb * NF : 0;            // first query tile that reaches this block's first key
    const int nqb = T / 64;
    // threads 0-15 move the tile's lse2, 16-31 its delta (one float4 each)
    const float* lsrc = tid < 16 ? L2 + 4 * tid : Dl + 4 * (tid - 16);
    float4 lrow = {0.f, 0.f, 0.f, 0.f};
    TileLd tq, tdo;
    tq.load(Q + (long)qb0 * 64 * ld, ld, tid);
    tdo.load(dOp + (long)qb0 * 64 * D, D, tid);
    if (tid < 32) lrow = *reinterpret_cast<const float4*>(lsrc + qb0 * 64);
    tq.store(smem[0][0], tid);
    tdo.store(smem[0][1], tid);
    if (tid < 32) *reinterpret_cast<float4*>(&lsd[0][tid >> 4][4 * (tid & 15)]) = lrow;
    // every prologue load (the K / V fragments above included) has landed: no wait for them inside the loop,
    // where the compiler's in-order vmcnt waits would otherwise also wait out the next tile's prefetch
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int qb = qb0; qb < nqb; ++qb) {
        const int cur = (qb - qb0) & 1;
        const bool more = qb + 1 < nqb;
        if (more) {
            tq.load(Q + (long)(qb + 1) * 64 * ld, ld, tid);
            tdo.load(dOp + (long)(qb + 1) * 64 * D, D, tid);
            if (tid < 32) lrow = *reinterpret_cast<const float4*>(lsrc + (qb + 1) * 64);
        }
        const int qs = qb * 64;
        if (!causal || qs + 63 >= k0) {
            const bf16_t* Qi = smem[cur][0];
            const bf16_t* Oi = smem[cur][1];
            // S[q][key], dP[q][key]: lane holds rows q = qs + 16 qi + 4 g + r, column key = k0 + 16 f + (lane & 15)
            f32x4_t s[NF][4], dp[NF][4];
#pragma unroll
            for (int qi = 0; qi < 4; ++qi) {
                const bf16x8_t q0f = frag_rows(Qi, 16 * qi, 0, lane), q1f = frag_rows(Qi, 16 * qi, 1, lane);
                const bf16x8_t o0f = frag_rows(Oi, 16 * qi, 0, lane), o1f = frag_rows(Oi, 16 * qi, 1, lane);
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    f32x4_t z = {0.f, 0.f, 0.f, 0.f};
                    z = mfma(q0f, kf[f][0], z);
                    s[f][qi] = mfma(q1f, kf[f][1], z);
                    f32x4_t y = {0.f, 0.f, 0.f, 0.f};
                    y = mfma(o0f, vf[f][0], y);
                    dp[f][qi] = mfma(o1f, vf[f][1], y);
                }
            }
            const bool diag = causal && qs < k0 + 16 * NF;  // wave-uniform: only these tiles need the mask
#pragma unroll
            for (int qi = 0; qi < 4; ++qi) {
                const int qr = qs + 16 * qi + 4 * g;
                const float4 lv = *reinterpret_cast<const float4*>(&lsd[cur][0][16 * qi + 4 * g]);
                const float4 dl = *reinterpret_cast<const float4*>(&lsd[cur][1][16 * qi + 4 * g]);
                const float la[4] = {lv.x, lv.y, lv.z, lv.w}, da[4] = {dl.x, dl.y, dl.z, dl.w};
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int kl = k0 + 16 * f + (lane & 15);
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[f][qi][r] = __builtin_amdgcn_exp2f(fmaf(s[f][qi][r], c, -la[r]));
                    if (diag) {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (kl > qr + r) s[f][qi][r] = 0.f;
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) dp[f][qi][r] = s[f][qi][r] * (dp[f][qi][r] - da[r]);
                }
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16x8_t pb[NF], sb[NF];
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    pb[f] = pack_acc(s[f][2 * kk], s[f][2 * kk + 1]);
                    sb[f] = pack_acc(dp[f][2 * kk], dp[f][2 * kk + 1]);
                }
                // all eight transposed fragments of this k-step issued before the MFMAs that use them (one at a
                // time, every MFMA waited out its own LDS read)
                bf16x8_t fo[4], fq[4];
#pragma unroll
                for (int df = 0; df < 4; ++df) {
                    fo[df] = frag_tr_perm(Oi, 16 * df, kk, lane);
                    fq[df] = frag_tr_perm(Qi, 16 * df, kk, lane);
                }
#pragma unroll
                for (int df = 0; df < 4; ++df)
#pragma unroll
                    for (int f = 0; f < NF; ++f) {
                        dv[f][df] = mfma(fo[df], pb[f], dv[f][df]);
                        dk[f][df] = mfma(fq[df], sb[f], dk[f][df]);
                    }
            }
        }
        if (more) {
            tq.store(smem[cur ^ 1][0], tid);
            tdo.store(smem[cur ^ 1][1], tid);
            if (tid < 32) *reinterpret_cast<float4*>(&lsd[cur ^ 1][tid >> 4][4 * (tid & 15)]) = lrow;
        }
        __syncthreads();
    }
    // lane holds dK^T / dV^T [d = 16 df + 4 g + r][key = kl]
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const int kl = k0 + 16 * f + (lane & 15);
        bf16_t* dkp = dqkv + ((long)b * T + kl) * ld + D + h * HD;
        bf16_t* dvp = dkp + D;
#pragma unroll
        for (int df = 0; df < 4; ++df) {
            u16x4_t a, v;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                a[r] = f2bf(dk[f][df][r] * scale);
                v[r] = f2bf(dv[f][df][r]);
            }
            *reinterpret_cast<u16x4_t*>(dkp + 16 * df + 4 * g) = a;
            *reinterpret_cast<u16x4_t*>(dvp + 16 * df + 4 * g) = v;
        }
    }
}

// dQ for 64 NF queries per block (wave w: NF 16-query fragments from q0 = 64 NF qb + 16 NF w); loop over 64-key
// tiles.  NF = 2 reads every K / V fragment out of LDS once for two query fragments: at NF = 1 a wave's 24 MFMAs
// per tile came with 24 KB of LDS reads, which saturated the LDS array (256 B/clk/CU) at the MFMA rate.
// DELTA: the block also forms delta = rowsum(dO . O) of its queries (the four 16-lane groups of a query row take
// 16 dims each) and writes it for attn_bwd_dkdv_kernel, which then runs after it: no separate delta launch
template <bool DELTA, int NF>
__global__ void __launch_bounds__(NTA) attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dO,
                                                          const float* __restrict__ lse2, float* __restrict__ delta,
                                                          const bf16_t* __restrict__ o,
                                                          bf16_t* __restrict__ dqkv, int T, int H, float scale,
                                                          int causal) {
    __shared__ __attribute__((aligned(16))) bf16_t smem[2][2][64 * HD];     // [buf][K|V]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
    const int nqb = T / (64 * NF);
    int qb, h, b;
    attn_block(nqb, H, true, qb, h, b);
    const int D = H * HD;
    const long ld = 3L * D;
    const bf16_t* Q = qkv + (long)b * T * ld + h * HD;
    const bf16_t* Kp = Q + D;
    const bf16_t* Vp = Q + 2 * D;
    const bf16_t* dOp = dO + (long)b * T * D + h * HD;
    const int q0 = qb * 64 * NF + 16 * NF * w;
    const float c = scale * LOG2E;
    int ql[NF];
    float lq[NF], dq_[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        ql[f] = q0 + 16 * f + (lane & 15);
        lq[f] = lse2[((long)b * H + h) * T + ql[f]];
        if constexpr (DELTA) {
            const long ro = ((long)b * T + ql[f]) * D + h * HD + 16 * g;
            float sd = 0.f;
#pragma unroll
            for (int c2 = 0; c2 < 2; ++c2) {
                float x[8], y[8];
                unpack8(*reinterpret_cast<const u16x8_t*>(o + ro + 8 * c2), x);
                unpack8(*reinterpret_cast<const u16x8_t*>(dO + ro + 8 * c2), y);
#pragma unroll
                for (int j = 0; j < 8; ++j) sd += x[j] * y[j];
            }
            sd = rsum4(sd);
            dq_[f] = sd;
            if (g == 0) delta[((long)b * H + h) * T + ql[f]] = sd;
        } else {
            dq_[f] = delta[((long)b * H + h) * T + ql[f]];
        }
    }

    bf16x8_t qf[NF][2], of[NF][2];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            qf[f][ks] = gfrag(Q + (long)(q0 + 16 * f) * ld, ld, ks, lane);
            of[f][ks] = gfrag(dOp + (long)(q0 + 16 * f) * D, D, ks, lane);
        }
    f32x4_t dq[NF][4];
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
        for (int i = 0; i < 4; ++i) dq[f][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int nkb = causal ? (qb + 1) * NF : T / 64;
    TileLd tk, tv;
    tk.load(Kp, ld, tid);
    tv.load(Vp, ld, tid);
    tk.store(smem[0][0], tid);
    tv.store(smem[0][1], tid);
    __syncthreads();
    for (int kb = 0; kb < nkb; ++kb) {
        const int cur = kb & 1;
        const bool more = kb + 1 < nkb;
        if (more) {
            tk.load(Kp + (long)(kb + 1) * 64 * ld, ld, tid);
            tv.load(Vp + (long)(kb + 1) * 64 * ld, ld, tid);
        }
        const int k0 = kb * 64;
        if (!causal || k0 <= q0 + 16 * NF - 1) {
            const bf16_t* Ki = smem[cur][0];
            const bf16_t* Vi = smem[cur][1];
            // S^T[key][q], dP^T[key][q]: lane holds rows key = k0 + 16 ki + 4 g + r, column q = ql[f]
            f32x4_t s[NF][4], dp[NF][4];
#pragma unroll
            for (int ki = 0; ki < 4; ++ki) {
                const bf16x8_t k0f = frag_rows(Ki, 16 * ki, 0, lane), k1f = frag_rows(Ki, 16 * ki, 1, lane);
                const bf16x8_t v0f = frag_rows(Vi, 16 * ki, 0, lane), v1f = frag_rows(Vi, 16 * ki, 1, lane);
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    f32x4_t z = {0.f, 0.f, 0.f, 0.f};
                    z = mfma(k0f, qf[f][0], z);
                    s[f][ki] = mfma(k1f, qf[f][1], z);
                    f32x4_t y = {0.f, 0.f, 0.f, 0.f};
                    y = mfma(v0f, of[f][0], y);
                    dp[f][ki] = mfma(v1f, of[f][1], y);
                }
            }
            const bool diag = causal && k0 + 63 > q0;     // wave-uniform: only these tiles need the mask
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
                for (int ki = 0; ki < 4; ++ki) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[f][ki][r] = __builtin_amdgcn_exp2f(fmaf(s[f][ki][r], c, -lq[f]));
                    if (diag) {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (k0 + 16 * ki + 4 * g + r > ql[f]) s[f][ki][r] = 0.f;
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) dp[f][ki][r] = s[f][ki][r] * (dp[f][ki][r] - dq_[f]);
                }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                bf16x8_t sb[NF];
#pragma unroll
                for (int f = 0; f < NF; ++f) sb[f] = pack_acc(dp[f][2 * kk], dp[f][2 * kk + 1]);
                bf16x8_t fk[4];                  // fragments issued before the MFMAs (as in attn_bwd_dkdv)
#pragma unroll
                for (int df = 0; df < 4; ++df) fk[df] = frag_tr_perm(Ki, 16 * df, kk, lane);
#pragma unroll
                for (int df = 0; df < 4; ++df)
#pragma unroll
                    for (int f = 0; f < NF; ++f) dq[f][df] = mfma(fk[df], sb[f], dq[f][df]);
            }
        }
        if (more) {
            tk.store(smem[cur ^ 1][0], tid);
            tv.store(smem[cur ^ 1][1], tid);
        }
        __syncthreads();
    }
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        bf16_t* dqp = dqkv + ((long)b * T + ql[f]) * ld + h * HD;
#pragma unroll
        for (int df = 0; df < 4; ++df) {
            u16x4_t a;
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = f2bf(dq[f][df][r] * scale);
            *reinterpret_cast<u16x4_t*>(dqp + 16 * df + 4 * g) = a;
        }
    }
}
}  // namespace

static dim3 attn_grid(int ntile, int H, int B) {
#if PDNN_ATTN_ORDER == 1
    return dim3(ntile * H * B);
#else
    return dim3(ntile, H, B);
#endif
}

// qkv [B*T][3*H*64] bf16 -> out [B*T][H*64] bf16, lse2 [B][H][T] fp32.  T % 128 == 0.
PDNN_API int pdnn_flash_attn_fwd(const bf16_t* qkv, bf16_t* out, float* lse2, int B, int T, int H, float scale,
                                 int causal, hipStream_t st) {
    if (T % 128) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(attn_fwd_kernel, attn_grid(T / 128, H, B), dim3(NTA), 0, st, qkv, out, lse2, T, H, scale, causal);
    PDNN_LAUNCH_RET;
}

static void launch_dkdv(const bf16_t* qkv, const bf16_t* dO, const float* lse2, const float* delta, bf16_t* dqkv, int B,
                        int T, int H, float scale, int causal, hipStream_t st) {
    if (pg::tune().attn_bwd_wide & 2)
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<2>, attn_grid(T / 128, H, B), dim3(NTA), 0, st, qkv, dO, lse2, delta,
                           dqkv, T, H, scale, causal);
    else
        hipLaunchKernelGGL(attn_bwd_dkdv_kernel<1>, attn_grid(T / 64, H, B), dim3(NTA), 0, st, qkv, dO, lse2, delta,
                           dqkv, T, H, scale, causal);
}

// dO [B*T][H*64], out/lse2 from the forward -> dqkv [B*T][3*H*64]; delta: fp32 [B][H][T] scratch.
PDNN_API int pdnn_flash_attn_bwd(const bf16_t* qkv, const bf16_t* out, const bf16_t* dO, const float* lse2,
                                 float* delta, bf16_t* dqkv, int B, int T, int H, float scale, int causal,
                                 hipStream_t st) {
    if (T % 128) return (int)hipErrorInvalidValue;
    const bool wq = pg::tune().attn_bwd_wide & 1;
    if (pg::tune().attn_delta_in_dq) {       // dQ first (it writes delta), then dK / dV
        if (wq)
            hipLaunchKernelGGL((attn_bwd_dq_kernel<true, 2>), attn_grid(T / 128, H, B), dim3(NTA), 0, st, qkv, dO, lse2,
                               delta, out, dqkv, T, H, scale, causal);
        else
            hipLaunchKernelGGL((attn_bwd_dq_kernel<true, 1>), attn_grid(T / 64, H, B), dim3(NTA), 0, st, qkv, dO, lse2,
                               delta, out, dqkv, T, H, scale, causal);
        launch_dkdv(qkv, dO, lse2, delta, dqkv, B, T, H, scale, causal, st);
        PDNN_LAUNCH_RET;
    }
    const long n = (long)B * T * H;
    hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((unsigned)((n + NTA - 1) / NTA)), dim3(NTA), 0, st, out, dO, delta,
                       B * T, T, H);
    launch_dkdv(qkv, dO, lse2, delta, dqkv, B, T, H, scale, causal, st);
    if (wq)
        hipLaunchKernelGGL((attn_bwd_dq_kernel<false, 2>), attn_grid(T / 128, H, B), dim3(NTA), 0, st, qkv, dO, lse2, delta,
                           out, dqkv, T, H, scale, causal);
    else
        hipLaunchKernelGGL((attn_bwd_dq_kernel<false, 1>), attn_grid(T / 64, H, B), dim3(NTA), 0, st, qkv, dO, lse2, delta,
                           out, dqkv, T, H, scale, causal);
    PDNN_LAUNCH_RET;
}
