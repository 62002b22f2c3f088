// MFMA implicit-GEMM engine for gfx950 (CDNA4): bf16 operands, fp32 accumulation.
//
// One templated kernel computes  C[m][n] = sum_k A(m,k) * B(n,k)  for every GEMM-shaped op of the
// framework:
//
//   op                      A operand (M x K)                    B operand (N x K)
//   linear fwd   Y=XW^T     X [M][K]            (A_KMAJOR)       W [N][K]           (B_KMAJOR)
//   linear dgrad dX=dY W    dY [M][N]           (A_KMAJOR)       W [N][K] as [k][n] (B_MNMAJOR)
//   linear wgrad dW=dY^T X  dY as [k=m][n]      (A_MNMAJOR)      X as [k=m][n]      (B_MNMAJOR)
//   conv fwd                im2col(In)          (A_CONV)         W [Ko][R][S][C]    (B_KMAJOR)
//   conv dgrad              col2im-gather(dOut) (A_CONVT)        W as [(r,s,ko)][c] (B_WT)
//   conv wgrad              dOut as [k=pix][ko] (A_MNMAJOR)      im2col(In) [pix][(r,s,c)] (B_IM2COL)
//
// (The reference computes these with cblas_dgemm / torch CPU ops: MPI_code/src/util/util.h:35-81,
//  MPI_code/src/nn/nn_layer.h:97-178, pytorch_code/model_ops/resnet.py:19-28.)
//
// Design (cdna_hip_programming.md §5):
//  * 256 threads = 4 waves in a 2x2 arrangement, block tile 128x128, K-step 64, every wave owns a
//    64x64 sub-tile = 4x4 `v_mfma_f32_16x16x32_bf16` fragments (16x16x32 holds a higher clock than
//    32x32x16 on random data: MI355X_MICROARCH.md DVFS item 7).
//  * Operands are staged global -> registers -> LDS (double buffered, one barrier per K-step, the
//    next tile's global loads issued before the MFMAs and written to LDS after them: T14).  Register
//    staging (not glds) because the conv loaders gather with zero-fill predicates and the optional
//    BN-affine+ReLU prologue transforms the data on its way to LDS.
//  * K-major LDS images (rows of 64 bf16 = 128 B) are read with ds_read_b128 through the XOR swizzle
//    chunk ^ ((row>>1)&7), which is conflict-free for the 16x16x32 fragment read pattern.
//    MN-major images ([k][mn] rows of 128 or 64 bf16) are read with the CDNA4 transpose read
//    `ds_read_b64_tr_b16` (T10) through a row-dependent even-chunk XOR that makes every 32-lane half
//    conflict-free.  That is how the reduction-major operands of the weight gradients reach MFMA
//    without any transpose pass over HBM.
//  * MFMA is issued with swapped operands (B fragment as src A) so each lane holds 4 consecutive
//    output columns; the epilogue stages the fp32 tile through LDS and writes 16-byte bf16 rows or
//    256-byte contiguous fp32 atomic rows (MI355X_MICROARCH.md "Global float atomics", access shape).
//  * Epilogue fusions: alpha, bias, ReLU, per-column BatchNorm partial statistics (sum, sum of
//    squares of the bf16-rounded outputs, one slab row per 64-row wave tile), or fp32 atomic
//    accumulation for split-K weight gradients.
//  * XCD-aware bijective block remap (T1) so neighbouring tiles share an XCD's L2.
#include "gemm_common.h"
#include "tuning.h"


namespace {
using namespace pg;

__device__ __forceinline__ u16x8_t zero8() {
    u16x8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
    return z;
}
__device__ __forceinline__ u16x8_t ldg16(const bf16_t* p) {
    return *reinterpret_cast<const u16x8_t*>(p);
}

__device__ __forceinline__ u16x8_t affine_relu8(u16x8_t v, const float* sc, const float* sh) {
    const float4 s0 = *reinterpret_cast<const float4*>(sc);
    const float4 s1 = *reinterpret_cast<const float4*>(sc + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(sh);
    const float4 h1 = *reinterpret_cast<const float4*>(sh + 4);
    const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    u16x8_t o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(fmaxf(fmaf(bf2f(v[j]), s[j], h[j]), 0.f));
    return o;
}

// ---------------------------------------------------------------------------------------------
// Operand loaders.  ROWS = the operand's tile extent along M (or N).  Every thread moves
// ROWS/32 16-byte chunks per K-step for both image kinds.
// ---------------------------------------------------------------------------------------------
// ---- K-major operands: row = tile row (m or n), 8 chunks of 8 k per row ----------------------
template <int ROWS, int KIND, bool PRO>   // KIND: 0 plain, 1 conv gather, 2 conv-transposed gather
struct KLoader {
    // The conv gathers resolve a chunk's source pixel once per TAP (r, s), not once per K-step: within a tap the
    // K-steps walk the channels of the same pixel, so a load is one add from the tap's pixel pointer.  Per-step
    // coordinate and 64-bit address math had made the stride-2 data gradients VALU-bound (23 vector instructions
    // per MFMA; rocprofv3 SQ_INSTS_VALU / SQ_INSTS_MFMA, gpurun_out/r4_29).
    static constexpr int NCH = ROWS / 32;
    const bf16_t* base[NCH];   // plain: row pointer; conv: image base pointer of the row's pixel
    const bf16_t* tp[NCH];     // conv: the row's source pixel for the current tap (valid when tv)
    int hb[NCH], wb[NCH];      // conv: top-left input coordinate of the row's window
    bool vrow[NCH], tv[NCH];
    int ch;                    // chunk column (fixed per thread)
    int r, s, c;               // conv: current (r, s, c) of this thread's chunk column
    int kcur;                  // current k of this thread's chunk

    __device__ __forceinline__ void retap(const GemmArgs& a) {
        const ConvGeom& g = a.g;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if constexpr (KIND == 1) {
                const int hi = hb[i] + r, wi = wb[i] + s;
                tv[i] = vrow[i] && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                tp[i] = base[i] + ((long)(tv[i] ? hi : 0) * g.W + (tv[i] ? wi : 0)) * g.C;
            } else if constexpr (KIND == 2) {
                int th = hb[i] - (g.r0 + g.st * r), tw = wb[i] - (g.s0 + g.st * s);
                bool v = vrow[i] && th >= 0 && tw >= 0;
                if (g.st == 2) {     // exact by construction of the parity class (negative: invalid anyway)
                    th >>= 1;
                    tw >>= 1;
                } else if (g.st != 1) {
                    th /= g.st;
                    tw /= g.st;
                }
                v = v && th < g.Ho && tw < g.Wo;
                tv[i] = v;
                tp[i] = base[i] + ((long)(v ? th : 0) * g.Wo + (v ? tw : 0)) * g.Ko;
            }
        }
    }
    __device__ __forceinline__ void derive_tap(const GemmArgs& a) {     // (r, s, c) of kcur
        const ConvGeom& g = a.g;
        if constexpr (KIND == 1) {
            const uint32_t rs = fdiv((uint32_t)kcur, g.dC);
            c = kcur - rs * g.C;
            r = fdiv(rs, g.dS);
            s = rs - r * g.S;
        } else if constexpr (KIND == 2) {     // r, s = tap indices within the parity class
            const uint32_t rs = fdiv((uint32_t)kcur, g.dKo);
            c = kcur - rs * g.Ko;
            r = fdiv(rs, g.dSc);
            s = rs - r * g.Sc;
        }
    }

    __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* ptr, long ld, int rows_total,
                                         int row0, int tid) {
        ch = tid & 7;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int row = row0 + (tid >> 3) + 32 * i;
            vrow[i] = row < rows_total;
            const int rr = vrow[i] ? row : 0;
            if constexpr (KIND == 0) {
                base[i] = ptr + (long)rr * ld;
            } else {
                const ConvGeom& g = a.g;
                // row -> (n, y, x) of the output grid (fwd: Ho x Wo; transposed: H x W of dIn)
                const uint32_t n = fdiv((uint32_t)rr, g.dHW);
                const uint32_t rem = (uint32_t)rr - n * g.dHW.d;
                const uint32_t y = fdiv(rem, g.dW);
                const uint32_t x = rem - y * g.dW.d;
                if constexpr (KIND == 1) {
                    hb[i] = (int)y * g.st - g.pad;
                    wb[i] = (int)x * g.st - g.pad;
                    base[i] = ptr + (long)n * g.H * g.W * g.C;
                } else {
                    hb[i] = (int)y * g.st + g.ph + g.pad;
                    wb[i] = (int)x * g.st + g.pw + g.pad;
                    base[i] = ptr + (long)n * g.Ho * g.Wo * g.Ko;
                }
            }
        }
        kcur = ch * 8;
        if constexpr (KIND != 0) {
            derive_tap(a);
            retap(a);
        }
    }
    __device__ __forceinline__ void seek(const GemmArgs& a, int k) {   // jump to K offset k (split-K)
        kcur = k + ch * 8;
        if constexpr (KIND != 0) {
            derive_tap(a);
            retap(a);
        }
    }
    __device__ __forceinline__ void load(const GemmArgs& a, int Ktot, u16x8_t* reg) {
        const bool kv = kcur < Ktot;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if constexpr (KIND == 0) {
                reg[i] = (vrow[i] && kv) ? ldg16(base[i] + kcur) : zero8();
            } else {
                u16x8_t x = (tv[i] && kv) ? ldg16(tp[i] + c) : zero8();
                if constexpr (KIND == 1 && PRO) {
                    if (tv[i] && kv) x = affine_relu8(x, a.pro_scale + c, a.pro_shift + c);
                }
                reg[i] = x;
            }
        }
    }
    __device__ __forceinline__ void advance(const GemmArgs& a) {
        kcur += BK;
        if constexpr (KIND != 0) {
            const int CC = KIND == 1 ? a.g.C : a.g.Ko;      // channels per tap
            if (CC >= BK) {          // CC % 64 == 0: at most one wrap (= one new tap) per K-step
                c += BK;
                if (c >= CC) {
                    c -= CC;
                    if (++s == (KIND == 1 ? a.g.S : a.g.Sc)) { s = 0; ++r; }
                    retap(a);
                }
            } else {                 // few channels (the 7x7 stem, C = 8): re-derive (r, s, c) every step
                derive_tap(a);
                retap(a);
            }
        }
    }
    __device__ __forceinline__ void store(bf16_t* img, const u16x8_t* reg, int tid) const {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int row = (tid >> 3) + 32 * i;
            *reinterpret_cast<u16x8_t*>(img + kimg_off(row, ch)) = reg[i];
        }
    }
};

// ---- MN-major operands: rows of the image are k, columns are m (or n) -------------------------
// KIND: 0 plain [k][ld] matrix, 1 weight-transposed gather (B_WT), 2 im2col of an NHWC tensor
template <int W, int KIND, bool PRO>
struct MLoader {
    static constexpr int CPR = W / 8;           // chunks per image row
    static constexpr int RPP = NT / CPR;        // image rows covered per pass
    static constexpr int NCH = 64 / RPP;        // = W / 32
    int ch, col;           // chunk column, global column index of this thread's chunk
    bool vcol;
    int krow0;             // first image row of this thread
    const bf16_t* ptr;
    long ld;
    // im2col: the column's (r, s, c) is fixed per block
    int cr, cs, cc;
    int kbase;
    float psc[PRO ? 8 : 1], psh[PRO ? 8 : 1];   // fused-prologue coefficients of this thread's 8 channels
    // weight gather (KIND 1): each chunk row's (ko, tap) and weight pointer, advanced incrementally (the per-step
    // two fast divisions and 64-bit address math per chunk were a large part of the VALU-bound stride-2 data
    // gradients, gpurun_out/r4_29)
    int wko[KIND == 1 ? NCH : 1], wrs[KIND == 1 ? NCH : 1];
    const bf16_t* wpt[KIND == 1 ? NCH : 1];

    __device__ __forceinline__ void wt_derive(const GemmArgs& a, int i) {
        const ConvGeom& g = a.g;
        const int k = kbase + krow0 + RPP * i;
        const uint32_t rs = fdiv((uint32_t)k, g.dKo);
        wko[i] = k - rs * g.Ko;
        wrs[i] = rs;
        wt_point(a, i);
    }
    __device__ __forceinline__ void wt_point(const GemmArgs& a, int i) {
        const ConvGeom& g = a.g;
        const uint32_t ir = fdiv((uint32_t)wrs[i], g.dSc);
        const int rr = g.r0 + g.st * (int)ir, ss = g.s0 + g.st * (int)(wrs[i] - ir * g.Sc);
        wpt[i] = ptr + ((long)wko[i] * g.R * g.S + rr * g.S + ss) * g.C + col;
    }

    __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld_, int cols_total,
                                         int col0, int tid) {
        ch = tid % CPR;
        krow0 = tid / CPR;
        col = col0 + ch * 8;
        vcol = col < cols_total;
        ptr = p;
        ld = ld_;
        kbase = 0;
        if constexpr (KIND == 1) {
#pragma unroll
            for (int i = 0; i < NCH; ++i) wt_derive(a, i);
        }
        if constexpr (KIND == 2) {
            const ConvGeom& g = a.g;
            const int cl = vcol ? col : 0;
            const uint32_t rs = fdiv((uint32_t)cl, g.dC);
            cc = cl - rs * g.C;
            cr = fdiv(rs, g.dS);
            cs = rs - cr * g.S;
            if constexpr (PRO) {   // the column (hence the channel) is fixed for the whole K loop
#pragma unroll
                for (int j = 0; j < 8; ++j) { psc[j] = a.pro_scale[cc + j]; psh[j] = a.pro_shift[cc + j]; }
            }
        }
    }
    __device__ __forceinline__ void seek(const GemmArgs& a, int k) {
        kbase = k;
        if constexpr (KIND == 1) {
#pragma unroll
            for (int i = 0; i < NCH; ++i) wt_derive(a, i);
        }
    }
    __device__ __forceinline__ void load(const GemmArgs& a, int Ktot, u16x8_t* reg) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int k = kbase + krow0 + RPP * i;
            const bool v = vcol && k < Ktot;
            if constexpr (KIND == 0) {
                reg[i] = v ? ldg16(ptr + (long)k * ld + col) : zero8();
            } else if constexpr (KIND == 1) {
                // reduction index k = (r*S + s)*Ko + ko ; weight W[ko][r][s][c], column = c (pointer kept by advance)
                reg[i] = v ? ldg16(wpt[i]) : zero8();
            } else {
                // reduction index k = output pixel (n, yo, xo); column = (r, s, c) of the input window
                const ConvGeom& g = a.g;
                const int kk = v ? k : 0;
                const uint32_t n = fdiv((uint32_t)kk, g.dHW);
                const uint32_t rem = (uint32_t)kk - n * g.dHW.d;
                const uint32_t yo = fdiv(rem, g.dW);
                const uint32_t xo = rem - yo * g.dW.d;
                const int hi = (int)yo * g.st - g.pad + cr, wi = (int)xo * g.st - g.pad + cs;
                const bool vv = v && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                u16x8_t x = vv ? ldg16(ptr + (((long)n * g.H + hi) * g.W + wi) * g.C + cc) : zero8();
                if constexpr (PRO) {
                    if (vv) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) x[j] = f2bf(fmaxf(fmaf(bf2f(x[j]), psc[j], psh[j]), 0.f));
                    }
                }
                reg[i] = x;
            }
        }
    }
    __device__ __forceinline__ void advance(const GemmArgs& a) {
        kbase += BK;
        if constexpr (KIND == 1) {
            const ConvGeom& g = a.g;
#pragma unroll
            for (int i = 0; i < NCH; ++i) {
                if (g.Ko >= BK) {         // at most one wrap into the next tap per K-step
                    wko[i] += BK;
                    if (wko[i] >= g.Ko) {
                        wko[i] -= g.Ko;
                        ++wrs[i];
                        wt_point(a, i);
                    } else {
                        wpt[i] += (long)BK * g.R * g.S * g.C;
                    }
                } else {
                    wt_derive(a, i);
                }
            }
        }
    }
    __device__ __forceinline__ void store(bf16_t* img, const u16x8_t* reg, int) const {
#pragma unroll
        for (int i = 0; i < NCH; ++i)
            *reinterpret_cast<u16x8_t*>(img + mimg_off<W>(krow0 + RPP * i, ch)) = reg[i];
    }
};

template <int AM, bool PRO> struct ASel;
template <bool PRO> struct ASel<A_KMAJOR, PRO> { using T = KLoader<128, 0, false>; static constexpr bool K = true; };
template <bool PRO> struct ASel<A_CONV, PRO> { using T = KLoader<128, 1, PRO>; static constexpr bool K = true; };
template <bool PRO> struct ASel<A_CONVT, PRO> { using T = KLoader<128, 2, false>; static constexpr bool K = true; };
template <bool PRO> struct ASel<A_MNMAJOR, PRO> { using T = MLoader<128, 0, false>; static constexpr bool K = false; };
template <bool PRO> struct ASel<A_IM2COL, PRO> { using T = MLoader<128, 2, PRO>; static constexpr bool K = false; };
template <int BMODE, bool PRO, int W> struct BSel;
template <bool PRO, int W> struct BSel<B_KMAJOR, PRO, W> { using T = KLoader<W, 0, false>; static constexpr bool K = true; };
template <bool PRO, int W> struct BSel<B_MNMAJOR, PRO, W> { using T = MLoader<W, 0, false>; static constexpr bool K = false; };
template <bool PRO, int W> struct BSel<B_WT, PRO, W> { using T = MLoader<W, 1, false>; static constexpr bool K = false; };
template <bool PRO, int W> struct BSel<B_IM2COL, PRO, W> { using T = MLoader<W, 2, PRO>; static constexpr bool K = false; };

constexpr int BMt = 128;
constexpr int CPAD = 4;                              // fp32 C-stage row padding (atomic epilogue only)
template <int BNW, int EM>
constexpr int smem_bytes() {
    const int ops = 2 * (BMt + BNW) * BK * 2;        // double-buffered A and B images
    const int cst = EM == E_ATOMIC ? BMt * (BNW + CPAD) * 4 : 0;
    return ops > cst ? ops : cst;
}


// BNW = block tile width (128, or 64 for the N <= 64 layers so no half-empty tiles are computed).
template <int AM, int BMODE, int EM, bool PRO_A, bool PRO_B, int BNW>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(GemmArgs a) {
    constexpr int WTN = BNW / 2, FN = WTN / 16;      // wave tile 64 x WTN, FN column fragments
    constexpr int BUF = (BMt + BNW) * BK;            // bf16 elements per (A|B) buffer
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const sbase = reinterpret_cast<bf16_t*>(smem);   // [buf][A 128x64 | B BNWx64]

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    if (gridDim.y > 1) {
        const int z = blockIdx.y, z1 = z / a.nb2, z2 = z - z1 * a.nb2;
        a.A += z1 * a.sA1 + z2 * a.sA2;
        a.B += z1 * a.sB1 + z2 * a.sB2;
        a.C = (void*)((char*)a.C + (z1 * a.sC1 + z2 * a.sC2) * (EM == E_BF16 ? 2 : 4));
        if (a.ep_res) a.ep_res += z1 * a.sC1 + z2 * a.sC2;
    }
    const int tiles_m = (a.M + BMt - 1) / BMt, tiles_n = (a.N + BNW - 1) / BNW;
    const int nwg = tiles_m * tiles_n;
    const int t = xcd_remap(blockIdx.x, nwg);
    // N fastest: consecutive tiles of one XCD share the same A rows (activations, the big operand).
    const int tm = t / tiles_n, tn = t % tiles_n;
    const int m0 = tm * BMt, n0 = tn * BNW;

    const int ktiles = (a.K + BK - 1) / BK;
    int kt0 = blockIdx.z * a.ktiles_per_split;
    int kt1 = min(ktiles, kt0 + a.ktiles_per_split);
    if (a.causal == 1 && n0 >= m0 + BMt) return;
    if (a.causal == 2) kt1 = min(kt1, (m0 + BMt + BK - 1) / BK);
    if (a.causal == 3) kt0 = max(kt0, m0 / BK);
    if (kt0 >= kt1) return;

    using LA = typename ASel<AM, PRO_A>::T;
    using LB = typename BSel<BMODE, PRO_B, BNW>::T;
    constexpr bool AK = ASel<AM, PRO_A>::K;
    constexpr bool BKm = BSel<BMODE, PRO_B, BNW>::K;
    LA la;
    LB lb;
    la.init(a, a.A, a.lda, a.M, m0, tid);
    lb.init(a, a.B, a.ldb, a.N, n0, tid);
    if (kt0) { la.seek(a, kt0 * BK); lb.seek(a, kt0 * BK); }

    u16x8_t ra[LA::NCH], rb[LB::NCH];
    f32x4_t acc[4][FN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    la.load(a, a.K, ra);
    lb.load(a, a.K, rb);
    la.store(sbase, ra, tid);
    lb.store(sbase + BMt * BK, rb, tid);

    int cur = 0;
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = kt + 1 < kt1;
        if (more) {   // issue the next tile's global loads before this tile's MFMAs (T14)
            la.advance(a);
            lb.advance(a);
            la.load(a, a.K, ra);
            lb.load(a, a.K, rb);
        }
        const bf16_t* A_ = sbase + cur * BUF;
        const bf16_t* B_ = A_ + BMt * BK;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8_t af[4], bfr[FN];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                if constexpr (AK) af[f] = frag_kmajor(A_, wm * 64 + f * 16 + (lane & 15), ks, lane);
                else af[f] = frag_mnmajor<128>(A_, wm * 64 + f * 16, ks, lane);
            }
#pragma unroll
            for (int f = 0; f < FN; ++f) {
                if constexpr (BKm) bfr[f] = frag_kmajor(B_, wn * WTN + f * 16 + (lane & 15), ks, lane);
                else bfr[f] = frag_mnmajor<BNW>(B_, wn * WTN + f * 16, ks, lane);
            }
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af[fm], acc[fm][fn], 0, 0, 0);
        }
        if (more) {   // write the next tile after the MFMAs, then one barrier
            bf16_t* nA = sbase + (cur ^ 1) * BUF;
            la.store(nA, ra, tid);
            lb.store(nA + BMt * BK, rb, tid);
        }
        __syncthreads();
        cur ^= 1;
    }

    // ---------------- epilogue ----------------
    // lane holds C[m = mb + (lane&15)][n = nb + 4*(lane>>4) + j] in acc[fm][fn][j]
    const int lm = lane & 15, lg = lane >> 4;

    if constexpr (EM == E_ATOMIC) {
        // stage the fp32 tile through LDS so every atomic wave-instruction covers 256 contiguous bytes
        float* cs = reinterpret_cast<float*>(smem);
        constexpr int LDC_S = BNW + CPAD;
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
                *reinterpret_cast<f32x4_t*>(cs + (wm * 64 + fm * 16 + lm) * LDC_S + wn * WTN + fn * 16 + 4 * lg) =
                    acc[fm][fn];
        __syncthreads();
        float* C = reinterpret_cast<float*>(a.C);
        if (a.transC) {
            // C is stored transposed (C^T[n][m], row stride ldc): each wave sweeps columns n, its lanes the
            // tile's 128 rows m -> 2 x 256 contiguous bytes per atomic wave-instruction
            for (int c = wave; c < BNW; c += 4) {
                const int n = n0 + c;
                if (n >= a.N) break;
#pragma unroll
                for (int h = 0; h < BMt / 64; ++h) {
                    const int r = lane + 64 * h;
                    const int m = m0 + r;
                    if (m < a.M) atomicAdd(C + (long)n * a.ldc + m, a.alpha * cs[r * LDC_S + c]);
                }
            }
            return;
        }
        for (int r = wave; r < BMt; r += 4) {
            const int m = m0 + r;
            if (m >= a.M) break;
#pragma unroll
            for (int h = 0; h < BNW / 64; ++h) {
                const int c = lane + 64 * h;
                const int n = n0 + c;
                if (n < a.N) atomicAdd(C + (long)m * a.ldc + n, a.alpha * cs[r * LDC_S + c]);
            }
        }
        return;
    } else {
        // One pass over the accumulators: alpha / bias / ReLU, optional residual add, then either
        //  (fwd)  per-column BN partial statistics of the bf16-rounded output, or
        //  (bwd)  BN-backward fusion: g -> gm = g * [t*mscale + mshift > 0] (the ReLU mask of the BN's
        //         output, recomputed from the BN input t), store gm, and per-column partials of
        //         sum(gm) and sum(gm * xhat), xhat = (t - mean) * invstd,
        // and direct register -> global stores (each lane writes 4 consecutive columns of one row).
        const bool bnb = a.ep_x != nullptr;
        const bool want_stats = EM == E_BF16 && (a.stats != nullptr);
        long orow[4];
        bool mv[4];
#pragma unroll
        for (int fm = 0; fm < 4; ++fm) {
            const int m = m0 + wm * 64 + fm * 16 + lm;
            mv[fm] = m < a.M;
            orow[fm] = m;
            if (a.scatter && mv[fm]) {
                const uint32_t nn = fdiv((uint32_t)m, a.g.dHW);
                const uint32_t rem = (uint32_t)m - nn * a.g.dHW.d;
                const uint32_t hc = fdiv(rem, a.g.dW);
                const uint32_t wc = rem - hc * a.g.dW.d;
                orow[fm] = ((long)nn * a.g.H + hc * a.g.st + a.g.ph) * a.g.W + wc * a.g.st + a.g.pw;
            }
        }
        // issue every epilogue load first so they are all in flight together (the kernel runs at low
        // occupancy; loads issued one fragment at a time would expose their full latency serially)
        u16x4_t rv[4][FN], tv[4][FN];
        if constexpr (EM == E_BF16) {
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn) {
                    const int n = n0 + wn * WTN + fn * 16 + 4 * lg;
                    const bool ok = mv[fm] && n + 4 <= a.N;
                    const long off = orow[fm] * a.ldc + n;
                    rv[fm][fn] = (a.ep_res && ok) ? *reinterpret_cast<const u16x4_t*>(a.ep_res + off) : u16x4_t{0, 0, 0, 0};
                    const bf16_t* tsrc = bnb ? a.ep_x : a.ep_dgelu;
                    tv[fm][fn] = (tsrc && ok) ? *reinterpret_cast<const u16x4_t*>(tsrc + off) : u16x4_t{0, 0, 0, 0};
                }
        }
        uint32_t pk[4][FN][2];     // packed bf16 results (2 dwords = 4 columns per lane and fragment)
        // per-column sums of every fragment column, stored after the loop: a statistics store inside it made the
        // next column's coefficient loads wait for it (s_waitcnt vmcnt counts stores too on gfx9)
        float ss[FN][4], qs[FN][4];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            const int n = n0 + wn * WTN + fn * 16 + 4 * lg;
            const bool nv = n < a.N, n4 = n + 4 <= a.N;
            float s[4] = {0, 0, 0, 0}, q[4] = {0, 0, 0, 0};
            float bmu[4], bis[4], bms[4], bmh[4];
            if (bnb && n4) {          // n % 4 == 0: 16-byte coefficient loads
                const float4 mu4 = *reinterpret_cast<const float4*>(a.ep_mean + n);
                const float4 is4 = *reinterpret_cast<const float4*>(a.ep_invstd + n);
                const float4 ms4 = *reinterpret_cast<const float4*>(a.ep_mscale + n);
                const float4 mh4 = *reinterpret_cast<const float4*>(a.ep_mshift + n);
                bmu[0] = mu4.x; bmu[1] = mu4.y; bmu[2] = mu4.z; bmu[3] = mu4.w;
                bis[0] = is4.x; bis[1] = is4.y; bis[2] = is4.z; bis[3] = is4.w;
                bms[0] = ms4.x; bms[1] = ms4.y; bms[2] = ms4.z; bms[3] = ms4.w;
                bmh[0] = mh4.x; bmh[1] = mh4.y; bmh[2] = mh4.z; bmh[3] = mh4.w;
            }
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
                const bool ok = mv[fm] && nv;
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[j] = acc[fm][fn][j] * a.alpha;
                    if (a.bias) v[j] += (n + j < a.N) ? a.bias[n + j] : 0.f;
                    if (a.relu == 1) v[j] = fmaxf(v[j], 0.f);
                }
                if constexpr (EM == E_BF16) {
                    if (a.relu == 2) {
                        if (a.ep_aux && ok) {
                            u16x4_t pre;
#pragma unroll
                            for (int j = 0; j < 4; ++j) pre[j] = f2bf(v[j]);
                            bf16_t* ax = a.ep_aux + orow[fm] * a.ldc + n;
                            if (n4) *reinterpret_cast<u16x4_t*>(ax) = pre;
                            else for (int j = 0; j < 4 && n + j < a.N; ++j) ax[j] = pre[j];
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(bf2f(f2bf(v[j])));
                    }
                    if (a.ep_dgelu) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] *= gelu_tanh_grad(bf2f(tv[fm][fn][j]));
                    }
                    if (a.ep_res) {
                        uint32_t mbits = 0xF;
                        if (a.ep_rmask && ok) {
                            const long off = orow[fm] * a.ldc + n;
                            mbits = a.ep_rmask[off >> 3] >> (off & 4);
                        }
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] += ((mbits >> j) & 1) ? bf2f(rv[fm][fn][j]) : 0.f;
                    }
                    if (bnb) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float t = bf2f(tv[fm][fn][j]);
                            const float gm = (ok && n4 && fmaf(t, bms[j], bmh[j]) > 0.f) ? bf2f(f2bf(v[j])) : 0.f;
                            v[j] = gm;
                            s[j] += gm;
                            q[j] += ok && n4 ? gm * (t - bmu[j]) * bis[j] : 0.f;
                        }
                    } else if (want_stats && ok) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float r = bf2f(f2bf(v[j]));
                            s[j] += r;
                            q[j] += r * r;
                        }
                    }
                    pk[fm][fn][0] = pk2bf(v[0], v[1]);
                    pk[fm][fn][1] = pk2bf(v[2], v[3]);
                } else {
                    if (!ok) continue;
                    float* C = reinterpret_cast<float*>(a.C) + orow[fm] * a.ldc + n;
                    if (n4 && (a.ldc & 3) == 0) {
                        *reinterpret_cast<float4*>(C) = make_float4(v[0], v[1], v[2], v[3]);
                    } else {
                        for (int j = 0; j < 4 && n + j < a.N; ++j) C[j] = v[j];
                    }
                }
            }
            if (want_stats) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {      // sum over the 16 rows (lanes l & 15) of the fragment column
                    ss[fn][j] = row16_sum(s[j]);
                    qs[fn][j] = row16_sum(q[j]);
                }
            }
        }
        if (want_stats) {
            const long row = (long)(a.stats_row0 + tm * 2 + wm) * 2;
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int n = n0 + wn * WTN + fn * 16 + 4 * lg;
                float* ps = stat_row(a.stats, row / 2, a.N) + n;
                stat_add_frag(ps, ps + a.N, lane, ss[fn], qs[fn], n + (lm & 3) < a.N);
            }
        }
        if constexpr (EM == E_BF16) {
          if (a.stage_store) {
            // Stage the bf16 tile through LDS ([128][BNW], 16-byte chunk c of row r at c ^ (r & 15): both
            // the 8-byte fragment writes and the 16-byte row reads are conflict-free), then every 16 (8)
            // threads write one full 256 (128)-byte row segment: whole cache lines per wave-instruction
            // instead of 64-byte pieces of 16 rows.
            constexpr int CPR = BNW / 8;                     // 16-byte chunks per tile row
            bf16_t* st = reinterpret_cast<bf16_t*>(smem);
            __syncthreads();                                 // operand images no longer read
#pragma unroll
            for (int fm = 0; fm < 4; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn) {
                    const int r = wm * 64 + fm * 16 + lm;
                    const int c = wn * WTN + fn * 16 + 4 * lg;
                    const int ch = (c >> 3) ^ (r & (CPR - 1));
                    *reinterpret_cast<uint2*>(st + r * BNW + ch * 8 + (c & 7)) = make_uint2(pk[fm][fn][0], pk[fm][fn][1]);
                }
            __syncthreads();
            constexpr int RPI = NT / CPR;                    // rows per pass
#pragma unroll
            for (int it = 0; it < BMt / RPI; ++it) {
                const int r = it * RPI + tid / CPR, j = tid % CPR;
                const int m = m0 + r;
                const int n = n0 + j * 8;
                if (m < a.M && n < a.N) {
                    long orw = m;
                    if (a.scatter) {
                        const uint32_t nn = fdiv((uint32_t)m, a.g.dHW);
                        const uint32_t rem = (uint32_t)m - nn * a.g.dHW.d;
                        const uint32_t hc = fdiv(rem, a.g.dW);
                        const uint32_t wc = rem - hc * a.g.dW.d;
                        orw = ((long)nn * a.g.H + hc * a.g.st + a.g.ph) * a.g.W + wc * a.g.st + a.g.pw;
                    }
                    const uint4 v = *reinterpret_cast<const uint4*>(st + r * BNW + ((j ^ (r & (CPR - 1))) << 3));
                    *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.C) + orw * a.ldc + n) = v;
                }
            }
          } else {
            // Lanes l, l+16, l+32, l+48 hold columns 0-3 / 4-7 / 8-11 / 12-15 of the same row.  One
            // permlane16_swap per dword between fragments (fn, fn+1) gives every lane 16 contiguous bytes:
            // 16-lane row g of the wave then holds fragment fn + (g & 1), columns 8*(g >> 1) .. +7.
            // Half the store instructions, 64-byte row segments (cdna_hip_programming.md T21, 16x16 form).
#pragma unroll
            for (int fm = 0; fm < 4; ++fm) {
#pragma unroll
                for (int fp = 0; fp < FN / 2; ++fp) {
                    const auto s0 = __builtin_amdgcn_permlane16_swap(pk[fm][2 * fp][0], pk[fm][2 * fp + 1][0], false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(pk[fm][2 * fp][1], pk[fm][2 * fp + 1][1], false, false);
                    const int n = n0 + wn * WTN + (2 * fp + (lg & 1)) * 16 + 8 * (lg >> 1);
                    if (mv[fm] && n + 8 <= a.N) {
                        uint4 o = make_uint4(s0[0], s1[0], s0[1], s1[1]);
                        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.C) + orow[fm] * a.ldc + n) = o;
                    } else if (mv[fm] && n < a.N) {
                        const uint32_t w4[4] = {s0[0], s1[0], s0[1], s1[1]};
                        bf16_t* C = reinterpret_cast<bf16_t*>(a.C) + orow[fm] * a.ldc + n;
                        for (int j = 0; j < 8 && n + j < a.N; ++j) C[j] = (bf16_t)(w4[j >> 1] >> (16 * (j & 1)));
                    }
                }
            }
          }
        }
    }
}

#include "gemm_glds.h"

// Engine selection (tuning.h entry glds: 0 off, 1 automatic, 2 whenever the operands allow).
// The 256-row tiles win once the grid fills most of the 256 CUs (>= 192 output tiles: r1 sweep,
// profiles/glds_threshold_sweep_r1.jsonl); with fewer tiles the 128-tile kernel's finer grid (2 blocks/CU) has
// better wave quantisation.  Per layer (profiles/conv_layers_glds_r1.json) glds wins the implicit-GEMM forward
// from a reduction of 1024 (512 / 1024 / never tied in r1) and the data gradient unless both C and K are small,
// but the glds data gradient's BN-backward epilogue tiles ran 2.3% slower in the whole step, so the data gradient
// stays on the register-staged kernel (7,790 -> 7,970 img/s).
constexpr int kGldsMinTiles = 192;
constexpr int kGldsFwdK = 1024;
int glds_mode() { return tune().glds; }
bool glds_enabled() { return glds_mode() != 0; }
template <int AM>
bool glds_worth(const GemmArgs& a, int batch, int splits) {
    if (glds_mode() == 2) return true;
    const long tiles = cdiv(a.M, GBM) * cdiv(a.N, glds_bn(a.N)) * (long)batch * splits;
    if (tiles < kGldsMinTiles) return false;
    if constexpr (AM == A_CONV) return a.K >= kGldsFwdK;
    if constexpr (AM == A_CONVT) return false;
    return true;
}

FastDiv make_fdiv(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}

// 1x1 stride-1 data gradients on the ping-pong engine: the plain / residual ones win there from K >= 512 with
// >= 128 output columns (r2_46: 512 vs 256 +0.5%); with the BN-backward epilogue (its BN input prefetched a
// fragment row ahead, gemm_pp.hip) from K >= 1024: ResNet-50 conv3 data gradients 65 / 51 vs 81 / 69 us in stages
// 3 / 4, but 111 vs 98 us at K = 512 (stage 2, N = 128: 3 rounds of 128-wide tiles; gpurun_out/r4_15).  The
// forward with BN statistics stays on the 128-row kernel; 1x1 convs the long-reduction kernel (conv1x1_wide.hip)
// takes are routed there first.
constexpr int kPPConvMinN = 128;
constexpr int kPPConvDgradK = 512;          // (with the BN epilogue: tuning pp_dgrad_bn_k)
// 128-row kernel bf16 epilogue: 1 = stores staged through LDS (full rows), 0 = direct fragment stores (tests)
int g_stage_store = 1;
int stage_store_mode() { return g_stage_store; }

template <int AM, int BMODE, int EM, bool PA, bool PB, int BNW>
int launch_w(const GemmArgs& a, int splits, hipStream_t st, int batch = 1) {
    static bool attr = false;
    constexpr int SM = smem_bytes<BNW, EM>();
    if (!attr) {
        attr = true;
        (void)hipFuncSetAttribute((const void*)gemm_kernel<AM, BMODE, EM, PA, PB, BNW>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, SM);
    }
    // a single K-step per block (K <= 64: the 1x1 "expand" convs) never touches the second operand
    // buffer: launch with half the LDS so twice as many blocks are resident per CU
    int sm = SM;
    if (a.ktiles_per_split <= 1 && EM != E_ATOMIC) sm = (BMt + BNW) * BK * 2;
    const int tiles = (int)(cdiv(a.M, BMt) * cdiv(a.N, BNW));
    dim3 grid(tiles, batch, splits);
    GemmArgs b = a;
    b.stage_store = stage_store_mode();
    hipLaunchKernelGGL((gemm_kernel<AM, BMODE, EM, PA, PB, BNW>), grid, dim3(NT), sm, st, b);
    PDNN_LAUNCH_RET;
}

// GEMMs of at most this many K-steps use the 128x64 tile (fewer registers: more blocks per CU to hide the
// load -> MFMA -> store latency of short reductions; r2_42-44 sweep: 24)
constexpr int kLowKBn64 = 24;

// the register-staged 128-row kernel only (the weight gradients' split-K atomics): N <= 64 -> 128x64 tile
template <int AM, int BMODE, int EM, bool PA, bool PB>
int launch_reg(const GemmArgs& a, int splits, hipStream_t st, int batch = 1) {
    if (a.N <= 64) return launch_w<AM, BMODE, EM, PA, PB, 64>(a, splits, st, batch);
    return launch_w<AM, BMODE, EM, PA, PB, 128>(a, splits, st, batch);
}

// glds engine when the operands allow it and the grid is big enough, else the 128-row kernel
template <int AM, int BMODE, int EM, bool PA, bool PB>
int launch(const GemmArgs& a, int splits, hipStream_t st, int batch = 1) {
    if constexpr (!PA && !PB && (AM == A_KMAJOR || AM == A_MNMAJOR) && (BMODE == B_KMAJOR || BMODE == B_MNMAJOR)) {
        if (pp_supported(a, AM, BMODE, EM, batch, splits)) return pp_launch(a, AM, BMODE, EM, st);
    }
    if constexpr (!PA && !PB) {
        if (glds_enabled() && glds_operands_ok<AM, BMODE>(a) && glds_worth<AM>(a, batch, splits)) {
            return launch_glds<AM, BMODE, EM>(a, splits, st, batch, glds_bn(a.N));
        }
    }
    if (a.N <= 64) return launch_w<AM, BMODE, EM, PA, PB, 64>(a, splits, st, batch);
    if (EM != E_ATOMIC && a.ktiles_per_split <= kLowKBn64)
        return launch_w<AM, BMODE, EM, PA, PB, 64>(a, splits, st, batch);
    return launch_w<AM, BMODE, EM, PA, PB, 128>(a, splits, st, batch);
}

template <int BNW>
int tiles_of(const GemmArgs& a) { return (int)(cdiv(a.M, BMt) * cdiv(a.N, BNW)); }

int pick_splits(const GemmArgs& a, int ktiles, int tiles, int max_splits) {
    // about one workgroup per CU, but keep >= 4 K-steps per split.  These are the atomic-epilogue weight
    // gradients (stride-2 3x3, the largest 1x1s) on the side stream: every split adds its tile into dW with
    // float atomics, so fewer splits mean fewer L2 atomics competing with the compute stream (ResNet-50 same
    // box: 256 vs 512 +0.3..+0.7% in 4 pairs, 384 equal, 128 -1.2..-1.8%, 1024 -0.2%; gpurun_out/r4_59-60;
    // the r2 sweep that chose 512 predates the two-stream schedule)
    const int blocks = 256;
    int want = (blocks + tiles - 1) / tiles;
    int s = want < max_splits ? want : max_splits;
    int cap = ktiles / 4;
    if (s > cap) s = cap;
    return s < 1 ? 1 : s;
}

void fill_geom(ConvGeom& g, int Nimg, int H, int W, int C, int Ho, int Wo, int R, int S, int st, int pad,
               int Ko) {
    g.Nimg = Nimg; g.H = H; g.W = W; g.C = C; g.Ho = Ho; g.Wo = Wo; g.R = R; g.S = S;
    g.st = st; g.pad = pad; g.Ko = Ko;
    g.dC = make_fdiv(C); g.dS = make_fdiv(S); g.dKo = make_fdiv(Ko);
    g.ph = g.pw = g.r0 = g.s0 = 0; g.Sc = S; g.dSc = make_fdiv(S);
}

// dst := src (or zeros when src is null), bf16 elements.  Used where a conv dgrad must pre-initialise
// dx before the parity-class GEMMs scatter into it: a kernel rather than hipMemsetAsync/hipMemcpyAsync
// keeps a training step a pure kernel sequence, which is what a captured hipGraph replays reliably
// (memset/memcpy graph nodes broke the second replay of a captured ResNet step).
__global__ void __launch_bounds__(256) copy_or_zero_kernel(bf16_t* __restrict__ dst, const bf16_t* __restrict__ src,
                                                           long n) {
    const long n8 = n >> 3;
    uint4* d8 = reinterpret_cast<uint4*>(dst);
    const uint4* s8 = reinterpret_cast<const uint4*>(src);
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long)gridDim.x * 256)
        d8[i] = src ? s8[i] : make_uint4(0u, 0u, 0u, 0u);
    for (long i = n8 * 8 + (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        dst[i] = src ? src[i] : (bf16_t)0;
}

}  // namespace

static void ensure_attrs() {}

// ------------------------------------------------------------------------------------------------
// C API
// ------------------------------------------------------------------------------------------------

PDNN_API int pdnn_set_staged_store(int mode) {
    const int old = g_stage_store;
    g_stage_store = mode;
    return old;
}

PDNN_API int pdnn_set_pp_mode(int mode) {
    int& m = pg::pp_mode_ref();
    const int old = m;
    m = mode;
    return old;
}

PDNN_API int pdnn_set_glds_mode(int mode) {
    const int old = glds_mode();
    tune().glds = mode;
    return old;
}

// Generic (batched) GEMM  C[M][N] = alpha * A . B  over nb1 x nb2 batches with two-level strides.
//   amode: 0 = A row-major [M][K] (K-major), 1 = A stored [K][M] (reduction-major)
//   bmode: 0 = B stored [N][K] (C = A.B^T),  1 = B stored [K][N]
//   out:   0 = bf16, 1 = fp32;  res (bf16, laid out like C) is added in the epilogue when given
//   causal: see GemmArgs::causal (0 for a dense GEMM)
PDNN_API int pdnn_gemm_batched(int amode, int bmode, int out_f32, const bf16_t* A, long lda, long sA1, long sA2,
                               const bf16_t* B, long ldb, long sB1, long sB2, void* C, long ldc, long sC1, long sC2,
                               int M, int N, int K, int nb1, int nb2, float alpha, const bf16_t* res,
                               int causal, hipStream_t st) {
    GemmArgs a{};
    a.causal = causal;
    a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.C = C; a.ldc = ldc;
    a.alpha = alpha; a.ep_res = res; a.ktiles_per_split = (int)cdiv(K, BK);
    a.nb2 = nb2 > 0 ? nb2 : 1;
    a.sA1 = sA1; a.sA2 = sA2; a.sB1 = sB1; a.sB2 = sB2; a.sC1 = sC1; a.sC2 = sC2;
    const int nb = (nb1 > 0 ? nb1 : 1) * a.nb2;
    const int key = amode * 100 + bmode * 10 + out_f32;
    switch (key) {
        case 0: return launch<A_KMAJOR, B_KMAJOR, E_BF16, false, false>(a, 1, st, nb);
        case 1: return launch<A_KMAJOR, B_KMAJOR, E_F32, false, false>(a, 1, st, nb);
        case 10: return launch<A_KMAJOR, B_MNMAJOR, E_BF16, false, false>(a, 1, st, nb);
        case 11: return launch<A_KMAJOR, B_MNMAJOR, E_F32, false, false>(a, 1, st, nb);
        case 110: return launch<A_MNMAJOR, B_MNMAJOR, E_BF16, false, false>(a, 1, st, nb);
        case 111: return launch<A_MNMAJOR, B_MNMAJOR, E_F32, false, false>(a, 1, st, nb);
        default: return (int)hipErrorInvalidValue;
    }
}

// Y[M][N] (bf16 or fp32) = alpha * X[M][K] . W[N][K]^T (+ bias) (relu)
PDNN_API int pdnn_gemm_nt(const bf16_t* X, long ldx, const bf16_t* W, long ldw, void* Y, long ldy,
                          int M, int N, int K, float alpha, const float* bias, int relu, int out_f32,
                          hipStream_t st) {
    ensure_attrs();
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K; a.A = X; a.lda = ldx; a.B = W; a.ldb = ldw; a.C = Y; a.ldc = ldy;
    a.alpha = alpha; a.bias = bias; a.relu = relu; a.ktiles_per_split = (int)cdiv(K, BK);
    return out_f32 ? launch<A_KMAJOR, B_KMAJOR, E_F32, false, false>(a, 1, st)
                   : launch<A_KMAJOR, B_KMAJOR, E_BF16, false, false>(a, 1, st);
}

// Y[M][N] = act(alpha * X[M][K] . W[N][K]^T + bias) (+ res); act 0/1/2 = none/ReLU/GELU; with GELU the
// pre-activation is also written to aux (same ld) for the backward.  dgelu: Y *= gelu'(dgelu) instead.
PDNN_API int pdnn_gemm_nt_ex(const bf16_t* X, long ldx, const bf16_t* W, long ldw, bf16_t* Y, long ldy,
                             int M, int N, int K, float alpha, const float* bias, int act, bf16_t* aux,
                             const bf16_t* res, const bf16_t* dgelu, int w_kn, hipStream_t st) {
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K; a.A = X; a.lda = ldx; a.B = W; a.ldb = ldw; a.C = Y; a.ldc = ldy;
    a.alpha = alpha; a.bias = bias; a.relu = act; a.ep_aux = aux; a.ep_res = res; a.ep_dgelu = dgelu;
    a.ktiles_per_split = (int)cdiv(K, BK);
    return w_kn ? launch<A_KMAJOR, B_MNMAJOR, E_BF16, false, false>(a, 1, st)
                : launch<A_KMAJOR, B_KMAJOR, E_BF16, false, false>(a, 1, st);
}

// FP8 GEMM (OCP e4m3 operands, both K-major [rows][K] bytes, K % 128 == 0, lda/ldb % 16 == 0):
// Y[M][N] = act(scale[0] * X . W^T + bias) (+ res), bf16 output (or fp32 with out_f32), optional BN
// statistics of the output.  Runs the glds engine on the block-scaled 16x16x128 MFMA (2x the bf16 rate)
// with unit block scales; `scale` (device) = 1 / (scale_x * scale_w).
PDNN_API int pdnn_gemm_fp8(const uint8_t* X, long ldx, const uint8_t* W, long ldw, void* Y, long ldy, int M, int N,
                           int K, const float* scale, const float* bias, int act, bf16_t* aux, const bf16_t* res,
                           float* stats, int out_f32, hipStream_t st) {
    if (K % 128 || ldx % 16 || ldw % 16 || N % 8 || M < 1) return (int)hipErrorInvalidValue;
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K / 2;
    a.A = reinterpret_cast<const bf16_t*>(X); a.lda = ldx / 2;
    a.B = reinterpret_cast<const bf16_t*>(W); a.ldb = ldw / 2;
    a.C = Y; a.ldc = ldy; a.alpha = 1.f; a.alpha_ptr = scale;
    a.bias = bias; a.relu = act; a.ep_aux = aux; a.ep_res = res; a.stats = stats;
    a.ktiles_per_split = (int)cdiv(a.K, BK);
    // ping-pong engine (fp8 slices of 128 bytes per row) unless tuning pp_fp8 = 0 / pp off: the glds engine
    if (pp_mode_ref() && M >= 16 && N >= 16)
        return pp_fp8_launch(a, out_f32 ? E_F32 : E_BF16, st);
    const int bn = glds_bn(N);
    if (out_f32) {
        if (bn == 256) return launch_glds_w<A_KMAJOR, B_KMAJOR, E_F32, 256, 1>(a, 1, st, 1);
        if (bn == 128) return launch_glds_w<A_KMAJOR, B_KMAJOR, E_F32, 128, 1>(a, 1, st, 1);
        return launch_glds_w<A_KMAJOR, B_KMAJOR, E_F32, 64, 1>(a, 1, st, 1);
    }
    if (bn == 256) return launch_glds_w<A_KMAJOR, B_KMAJOR, E_BF16, 256, 1>(a, 1, st, 1);
    if (bn == 128) return launch_glds_w<A_KMAJOR, B_KMAJOR, E_BF16, 128, 1>(a, 1, st, 1);
    return launch_glds_w<A_KMAJOR, B_KMAJOR, E_BF16, 64, 1>(a, 1, st, 1);
}

// Y[M][N] = alpha * X[M][K] . W[K][N]     (W row-major [K][N]: reduction-major B)
PDNN_API int pdnn_gemm_nn(const bf16_t* X, long ldx, const bf16_t* W, long ldw, void* Y, long ldy,
                          int M, int N, int K, float alpha, int out_f32, hipStream_t st) {
    ensure_attrs();
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K; a.A = X; a.lda = ldx; a.B = W; a.ldb = ldw; a.C = Y; a.ldc = ldy;
    a.alpha = alpha; a.ktiles_per_split = (int)cdiv(K, BK);
    return out_f32 ? launch<A_KMAJOR, B_MNMAJOR, E_F32, false, false>(a, 1, st)
                   : launch<A_KMAJOR, B_MNMAJOR, E_BF16, false, false>(a, 1, st);
}

// Cf32[M][N] += alpha * X[K][M]^T . Y[K][N]   (both reduction-major; split-K fp32 atomics).
// Cf32 must be initialised by the caller (zero for a fresh gradient).
PDNN_API int pdnn_gemm_tn_acc(const bf16_t* X, long ldx, const bf16_t* Y, long ldy, float* C, long ldc,
                              int M, int N, int K, float alpha, hipStream_t st) {
    ensure_attrs();
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K; a.A = X; a.lda = ldx; a.B = Y; a.ldb = ldy; a.C = C; a.ldc = ldc;
    a.alpha = alpha;
    const int ktiles = (int)cdiv(K, BK);
    a.ktiles_per_split = ktiles;
    if (glds_enabled() && glds_operands_ok<A_MNMAJOR, B_MNMAJOR>(a)) {
        const int bn = glds_bn(N);
        const int tiles = (int)(cdiv(M, GBM) * cdiv(N, bn));
        if (tiles >= 192 || glds_mode() == 2) {   // enough output tiles: split K only until the grid covers the CUs once
            int s = (256 + tiles - 1) / tiles;
            s = s < ktiles / 4 ? s : ktiles / 4;
            s = s < 1 ? 1 : s;
            a.ktiles_per_split = (int)cdiv(ktiles, s);
            return launch_glds<A_MNMAJOR, B_MNMAJOR, E_ATOMIC>(a, (int)cdiv(ktiles, a.ktiles_per_split), st, 1, bn);
        }
    }
    const int tiles = N <= 64 ? tiles_of<64>(a) : tiles_of<128>(a);
    const int splits = pick_splits(a, ktiles, tiles, 256);
    a.ktiles_per_split = (int)cdiv(ktiles, splits);
    return launch_w<A_MNMAJOR, B_MNMAJOR, E_ATOMIC, false, false, 128>(a, (int)cdiv(ktiles, a.ktiles_per_split), st);
}

// Convolution forward, NHWC bf16 activations, weight [Ko][R][S][C] bf16 (== torch channels_last).
// Optional fused prologue relu(x*scale[c]+shift[c]) on the input, optional BN partial statistics
// of the output (stats: [2*ceil(M/128)*2][N] floats, see pdnn_bn_stats_finalize).
PDNN_API int pdnn_conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int Nimg, int H, int W, int C,
                           int Ko, int R, int S, int st, int pad, int Ho, int Wo,
                           const float* pro_scale, const float* pro_shift, float* stats,
                           hipStream_t stream) {
    ensure_attrs();
    GemmArgs a{};
    a.M = Nimg * Ho * Wo; a.N = Ko; a.K = R * S * C;
    a.A = x; a.B = w; a.ldb = (long)R * S * C; a.C = y; a.ldc = Ko; a.alpha = 1.f;
    fill_geom(a.g, Nimg, H, W, C, Ho, Wo, R, S, st, pad, Ko);
    a.g.dHW = make_fdiv(Ho * Wo); a.g.dW = make_fdiv(Wo);
    a.pro_scale = pro_scale; a.pro_shift = pro_shift; a.stats = stats;
    a.ktiles_per_split = (int)cdiv(a.K, BK);
    if (R == 1 && S == 1 && st == 1 && pad == 0 && !pro_scale && C >= tune().pp_conv_fwd_c) {
        // 1x1 stride-1 without a prologue is the plain GEMM y[P][Ko] = x[P][C] . w[Ko][C]^T: the ping-pong engine
        // with its statistics epilogue (ResNet-50's conv1 / shortcut forwards with C >= 512)
        GemmArgs p{};
        p.M = a.M; p.N = Ko; p.K = C;
        p.A = x; p.lda = C; p.B = w; p.ldb = C; p.C = y; p.ldc = Ko; p.alpha = 1.f; p.stats = stats;
        if (pp_supported(p, A_KMAJOR, B_KMAJOR, E_BF16, 1, 1)) return pp_launch(p, A_KMAJOR, B_KMAJOR, E_BF16, stream);
    }
    if (pro_scale) return launch<A_CONV, B_KMAJOR, E_BF16, true, false>(a, 1, stream);
    return launch<A_CONV, B_KMAJOR, E_BF16, false, false>(a, 1, stream);
}

// Convolution data gradient: dx[N][H][W][C] = sum over (r, s, ko) dy[...] * w[ko][r][s][c].
// stride > 1 is decomposed into st*st parity classes of dx pixels; each class is a dense implicit GEMM
// over only the taps that reach it (no MFMA work on the zero-stuffed positions of the transposed conv).
struct DgradClass { int ph, pw, r0, s0, Rc, Sc, Hc, Wc; };
static int dgrad_classes(int H, int W, int R, int S, int st, int pad, DgradClass* out, bool* any_empty) {
    int n = 0;
    *any_empty = false;
    for (int ph = 0; ph < st; ++ph)
        for (int pw = 0; pw < st; ++pw) {
            DgradClass c;
            c.ph = ph; c.pw = pw;
            c.r0 = (ph + pad) % st; c.s0 = (pw + pad) % st;
            c.Rc = c.r0 < R ? (R - c.r0 + st - 1) / st : 0;
            c.Sc = c.s0 < S ? (S - c.s0 + st - 1) / st : 0;
            c.Hc = ph < H ? (H - ph + st - 1) / st : 0;
            c.Wc = pw < W ? (W - pw + st - 1) / st : 0;
            if (c.Hc * c.Wc == 0) continue;
            if (c.Rc * c.Sc == 0) { *any_empty = true; continue; }
            out[n++] = c;
        }
    return n;
}

// Number of stats wave-rows (slab rows / 2) the fused dgrad epilogue writes.
PDNN_API int pdnn_conv_dgrad_stats_rows(int Nimg, int H, int W, int R, int S, int st, int pad) {
    DgradClass cl[16];
    bool e;
    const int n = dgrad_classes(H, W, R, S, st, pad, cl, &e);
    int rows = 0;
    for (int i = 0; i < n; ++i) rows += (int)cdiv((long)Nimg * cl[i].Hc * cl[i].Wc, BMt) * 2;
    return rows;
}

// Convolution data gradient: dx[N][H][W][C] = sum over (r, s, ko) dy[...] * w[ko][r][s][c] (+ res).
// stride > 1 is decomposed into st*st parity classes of dx pixels; each class is a dense implicit GEMM
// over only the taps that reach it (no MFMA work on the zero-stuffed positions of the transposed conv).
// Optional epilogue fusions: `res` is added to dx; with `bn_x` the output is the BN-backward masked
// gradient gm = dx * [bn_x*mscale + mshift > 0] and `stats` receives the partial sums of gm and
// gm * (bn_x - mean) * invstd (the BatchNorm backward reduction, see batchnorm.hip).
PDNN_API int pdnn_conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int Nimg, int H, int W, int C,
                             int Ko, int R, int S, int st, int pad, int Ho, int Wo, float* stats,
                             const bf16_t* res, const uint8_t* res_mask, const bf16_t* bn_x, const float* bn_mean,
                             const float* bn_invstd, const float* bn_mscale, const float* bn_mshift,
                             hipStream_t stream) {
    if (res_mask && (st != 1 || C % 8 || !res || res == dx)) return (int)hipErrorInvalidValue;
    ensure_attrs();
    if (R == 1 && S == 1 && st == 1 && pad == 0 && C >= kPPConvMinN && Ko >= (bn_x ? tune().pp_dgrad_bn_k : kPPConvDgradK)) {
        // 1x1 stride-1: dx[M][C] = dy[M][Ko] . w[Ko][C] (w as a [k][n] matrix) on the ping-pong engine
        GemmArgs a{};
        a.M = Nimg * H * W; a.N = C; a.K = Ko;
        a.A = dy; a.lda = Ko; a.B = w; a.ldb = C; a.C = dx; a.ldc = C; a.alpha = 1.f; a.stats = stats;
        a.ep_res = res; a.ep_rmask = res_mask;
        a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
        if (pp_supported(a, A_KMAJOR, B_MNMAJOR, E_BF16, 1, 1)) return pp_launch(a, A_KMAJOR, B_MNMAJOR, E_BF16, stream);
    }
    if (R == 1 && S == 1 && st == 2 && pad == 0 && !bn_x && !res_mask && (res == dx || !res) &&
        C >= kPPConvMinN && Ko >= kPPConvDgradK) {
        // 1x1 stride-2 (the ResNet shortcut) accumulated in place: one parity class, whose GEMM rows are dy's
        // pixels as they are (A plain K-major), scattered to the even pixels of dx by the ping-pong epilogue
        // (with res == dx the odd pixels keep dx); 180 / 145 / 135 us on the 128-row engine's gather before
        GemmArgs a{};
        a.M = Nimg * Ho * Wo; a.N = C; a.K = Ko;
        a.A = dy; a.lda = Ko; a.B = w; a.ldb = C; a.C = dx; a.ldc = C; a.alpha = 1.f;
        a.ep_res = res;
        fill_geom(a.g, Nimg, H, W, C, Ho, Wo, R, S, st, pad, Ko);
        a.g.dHW = make_fdiv(Ho * Wo); a.g.dW = make_fdiv(Wo);
        a.scatter = 1;
        if (res == dx && pp_supported(a, A_KMAJOR, B_MNMAJOR, E_BF16, 1, 1))
            return pp_launch(a, A_KMAJOR, B_MNMAJOR, E_BF16, stream);
    }
    DgradClass cl[16];
    bool any_empty;
    const int ncl = dgrad_classes(H, W, R, S, st, pad, cl, &any_empty);
    if (any_empty && !(res == dx && !bn_x)) {   // pixels no tap reaches: zero (or the residual, unless in place)
        const long n = (long)Nimg * H * W * C;         // C % 8 == 0: 16-B aligned rows
        hipLaunchKernelGGL(copy_or_zero_kernel, dim3(stream_grid(n / 8 + 1, 256)), dim3(256), 0, stream, dx,
                           (res && !bn_x) ? res : nullptr, n);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return (int)e;
    }
    int row0 = 0;
    for (int i = 0; i < ncl; ++i) {
        const DgradClass& c = cl[i];
        GemmArgs a{};
        a.M = Nimg * c.Hc * c.Wc; a.N = C; a.K = c.Rc * c.Sc * Ko;
        a.A = dy; a.B = w; a.C = dx; a.ldc = C; a.alpha = 1.f; a.stats = stats;
        fill_geom(a.g, Nimg, H, W, C, Ho, Wo, R, S, st, pad, Ko);
        a.g.ph = c.ph; a.g.pw = c.pw; a.g.r0 = c.r0; a.g.s0 = c.s0; a.g.Sc = c.Sc; a.g.dSc = make_fdiv(c.Sc);
        a.g.dHW = make_fdiv(c.Hc * c.Wc); a.g.dW = make_fdiv(c.Wc);
        a.scatter = st > 1;
        a.stats_row0 = row0;
        a.ep_res = res; a.ep_rmask = res_mask;
        a.ep_x = bn_x; a.ep_mean = bn_mean; a.ep_invstd = bn_invstd; a.ep_mscale = bn_mscale; a.ep_mshift = bn_mshift;
        a.ktiles_per_split = (int)cdiv(a.K, BK);
        const int rc = launch<A_CONVT, B_WT, E_BF16, false, false>(a, 1, stream);
        if (rc) return rc;
        row0 += (int)cdiv(a.M, BMt) * 2;
    }
    return 0;
}

// Convolution weight gradient (accumulating into fp32 dw[Ko][R][S][C]): split-K over output pixels.
PDNN_API int pdnn_conv_wgrad(const bf16_t* x, const bf16_t* dy, float* dw, int Nimg, int H, int W, int C,
                             int Ko, int R, int S, int st, int pad, int Ho, int Wo,
                             const float* pro_scale, const float* pro_shift, hipStream_t stream) {
    ensure_attrs();
    GemmArgs a{};
    const bool swap = Ko <= 64 && R * S * C >= 128;   // put the small Ko dimension on the 64-wide N tile
    a.K = Nimg * Ho * Wo;
    if (swap) {   // dW^T[(r,s,c)][ko] = im2col(x)^T . dy  -> stored transposed into dw[ko][(r,s,c)]
        a.M = R * S * C; a.N = Ko;
        a.A = x; a.B = dy; a.ldb = Ko; a.transC = 1;
    } else {      // dW[ko][(r,s,c)] = dy^T . im2col(x)
        a.M = Ko; a.N = R * S * C;
        a.A = dy; a.lda = Ko; a.B = x;
    }
    a.C = dw; a.ldc = (long)R * S * C; a.alpha = 1.f;
    fill_geom(a.g, Nimg, H, W, C, Ho, Wo, R, S, st, pad, Ko);
    a.g.dHW = make_fdiv(Ho * Wo); a.g.dW = make_fdiv(Wo);
    a.pro_scale = pro_scale; a.pro_shift = pro_shift;
    const int ktiles = (int)cdiv(a.K, BK);
    if (!pro_scale && glds_mode() == 2 &&      // measured slower than the 128-row kernel: forced mode only
        (swap ? glds_operands_ok<A_IM2COL, B_MNMAJOR>(a) : glds_operands_ok<A_MNMAJOR, B_IM2COL>(a))) {
        // glds engine: split the pixel reduction so ~1.5 blocks per CU run, >= 8 K-steps each
        const int bn = glds_bn(a.N);
        const int tiles = (int)(cdiv(a.M, GBM) * cdiv(a.N, bn));
        int sp = (384 + tiles - 1) / tiles;
        sp = sp < ktiles / 8 ? sp : ktiles / 8;
        sp = sp < 1 ? 1 : sp;
        a.ktiles_per_split = (int)cdiv(ktiles, sp);
        const int nz = (int)cdiv(ktiles, a.ktiles_per_split);
        if (swap) return launch_glds<A_IM2COL, B_MNMAJOR, E_ATOMIC>(a, nz, stream, 1, bn);
        return launch_glds<A_MNMAJOR, B_IM2COL, E_ATOMIC>(a, nz, stream, 1, bn);
    }
    const int tiles = a.N <= 64 ? tiles_of<64>(a) : tiles_of<128>(a);
    const int splits = pick_splits(a, ktiles, tiles, 1024);
    a.ktiles_per_split = (int)cdiv(ktiles, splits);
    const int nz = (int)cdiv(ktiles, a.ktiles_per_split);
    if (swap) {
        if (pro_scale) return launch_reg<A_IM2COL, B_MNMAJOR, E_ATOMIC, true, false>(a, nz, stream);
        return launch_reg<A_IM2COL, B_MNMAJOR, E_ATOMIC, false, false>(a, nz, stream);
    }
    if (pro_scale) return launch_reg<A_MNMAJOR, B_IM2COL, E_ATOMIC, false, true>(a, nz, stream);
    return launch_reg<A_MNMAJOR, B_IM2COL, E_ATOMIC, false, false>(a, nz, stream);
}

// Number of stats rows the fused epilogue writes for M output rows (2 wave-rows per 128-row tile).
PDNN_API int pdnn_gemm_stats_rows(int M) { return (int)cdiv(M, BMt) * 2; }
