// Ping-pong GEMM engine ("pp") for gfx950: the plain-GEMM kernel of the transformer linears and other
// large dense GEMMs (reference GEMM sites MPI_code/src/util/util.h:35-81,
// MPI_code/src/nn/nn_layer.h:111-175).
//
//  * Block tile 256 x BN, 512 threads = 8 waves in two GROUPS of four: group g owns output rows
//    [128 g, 128 g + 128); its four waves form a WR x WC grid over that 128 x BN block.  Waves w and w + 4
//    share a SIMD, so every SIMD holds one wave of each group.
//  * The groups run the same program shifted by one barrier (group 1 executes one extra s_barrier before
//    its loop, group 0 one after): while a wave of one group issues its MFMAs, its partner on the same
//    SIMD reads the fragments of the next K-slice from LDS and issues global->LDS copies further ahead,
//    so one wave's matrix work covers its partner's load latency (cdna_hip_programming.md §5 "256²
//    8-phase template", MI355X_MICROARCH.md "Two waves per SIMD").
//  * K is consumed in slices of 32.  A slice of both operands ((256 + BN) x 32 bf16) is staged by
//    `global_load_lds_dwordx4` (glds) into a ring of NB slots; each group copies its half of every slice.
//    A slice is issued NB-1 slices ahead and retired with a COUNTED `s_waitcnt vmcnt(N)` in the load
//    segment before its first reader (never vmcnt(0) in the steady state); only raw `s_barrier`s are
//    used, so the copies stay in flight across barriers ("Pipelining across barriers"; all LDS is the
//    one dynamic array, so hipcc inserts no vmcnt(0) of its own — checked in the .s).
//      RAW: slice s+1 is retired by each group in its load segment of slice s, one barrier before the
//           other group's first read of it.
//      WAR: slot (s-1) mod NB is refilled in the load segment of slice s; both groups read slice s-1 in
//           earlier load segments that end with `s_waitcnt lgkmcnt(0)` before their barrier.
//  * LDS images: K-major operands [rows][32] bf16 (64-byte rows, 16-byte chunk c of row r stored at
//    c ^ t[(r >> 2) & 3], t = {0, 2, 3, 1}: conflict-free for the four 16-lane groups of ds_read_b128);
//    MN-major operands (BN = 128 / 256 only) [32 k-rows][W] read with `ds_read_b64_tr_b16`.  glds writes
//    lane-linear images, so the swizzle is applied to the per-lane GLOBAL source address (rule 21).
//  * Tile widths 96 / 128 / 192 / 256 / 288 so that the grid fills the 256 CUs in whole rounds for the
//    GPT-2 shapes (M = 8192 tokens: N = 768 -> 256x96 = 256 tiles, 2304 -> 256x288 = 256, 3072 -> 256x192
//    = 512); the host picks the width with the smallest rounds x tile-time estimate.
//  * Tile order: XCD-aware bijective remap (T1), then groups of 4 tile rows so the 32 tiles an XCD runs
//    at once share 4 A row-blocks and 8 B column-blocks in its L2.
//  * MFMA v_mfma_f32_16x16x32_bf16 with swapped operands, so each lane ends with 4 consecutive output
//    columns; bf16 epilogues pair fragments with permlane16 swaps into 16-byte stores (T21).
//  * Epilogues: alpha, bias, ReLU / GELU (+ pre-activation to ep_aux), dGELU, residual add (bf16);
//    fp32 store / in-place accumulate (acc_c) / split-K partial slabs (slab reduction kernel below).
#include "gemm_common.h"
#include "tuning.h"

namespace pg {
namespace {

constexpr int PP_BM = 256;
constexpr int PP_SK = 32;                 // K depth of one slice
constexpr int PP_GROUP = 4;               // tile rows per L2 group

// fusion flags (gemm_pp_kernel FX)
constexpr int FX_PRO = 1;      // A := relu(A * pro_scale[k] + pro_shift[k])  (K-major A, no split-K, K <= PP_PRO_MAXK)
// (FX_PRO keeps the scale/shift table in LDS behind the ring; FX_BNB keeps mscale/mshift there, N <= PP_PRO_MAXK)
constexpr int FX_STATS = 2;    // per-column (sum, sum of squares) of the bf16 output, one slab row pair per 64 rows
constexpr int FX_BNB = 4;      // output gm = v * [ep_x*mscale + mshift > 0]; slab gets sum gm, sum gm*xhat
constexpr int PP_PRO_MAXK = 1024;

// DT = 2: bf16 with 64-deep slices (128-byte rows: one 128-byte L2 request per row and slice where 32-deep slices
// issue two 64-byte ones; the N = 768 GEMMs issued 2.1x hipBLASLt's TCP->TCC read requests, gpurun_out/r5_17).
// DT = 1: fp8 (OCP e4m3) operands, both K-major, every K / ld in units of 2 fp8 (the loaders move bytes);
// a slice is then 64 units = 128 fp8 per row, consumed by one block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// per fragment pair (unit block scales; the per-tensor scales come in through alpha_ptr).
template <int BN_, int WR_, int NB_, int DT_ = 0>
struct PPC {
    static constexpr int BN = BN_, WR = WR_, WC = 4 / WR_, NB = NB_, DT = DT_;
    static constexpr int SK = DT ? 64 : PP_SK;            // slice depth in bf16 units
    static constexpr int WTM = 128 / WR, WTN = BN / WC;
    static constexpr int FM = WTM / 16, FN = WTN / 16;
    static constexpr int IMA = PP_BM * SK, IMB = BN * SK, SLOT = IMA + IMB;
    static constexpr int SMEM = NB * SLOT * 2;
    static_assert(WTN % 16 == 0 && WTM % 16 == 0, "wave tile");
    static_assert(SMEM <= 160 * 1024, "LDS");
};

__device__ __forceinline__ int pp_swz(int row) { return (0x78 >> (((row >> 2) & 3) << 1)) & 3; }
__device__ __forceinline__ int pp_koff(int row, int chunk) { return row * PP_SK + ((chunk ^ pp_swz(row)) << 3); }

typedef __attribute__((ext_vector_type(8))) int v8i_t;
typedef __attribute__((ext_vector_type(4))) int v4i_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2_t;
// fp8 fragment of the 16x16x128 MFMA from a 128-byte-row image: lane l holds k-bytes [32 (l >> 4), +32)
// of its row = 16-byte chunks 2g, 2g + 1 (g = l >> 4)
__device__ __forceinline__ v8i_t frag8(const bf16_t* img, int row, int lane) {
    const int g = lane >> 4;
    const v4i_t lo = *reinterpret_cast<const v4i_t*>(img + kimg_off(row, 2 * g));
    const v4i_t hi = *reinterpret_cast<const v4i_t*>(img + kimg_off(row, 2 * g + 1));
    return v8i_t{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// One operand's copies: NR = ROWS/16 wave-instructions of 1 KiB per slice, spread over the 8 waves
// (NI each; instructions past NR duplicate the last one: identical bytes to identical LDS addresses).
//   K-major  [rows][K]: instruction j covers rows 16 j .. 16 j + 15 (lane: row 16 j + lane / 4, chunk lane & 3)
//   MN-major [K][cols]: instruction j covers k-rows RPI j .. RPI j + RPI - 1, RPI = 512 / ROWS
template <int ROWS, bool KMAJ, int SK = PP_SK>
struct PPLoader {
    static_assert(SK == PP_SK || KMAJ, "128-byte slices: K-major operands only");
    // SK = 64 (fp8): 128-byte rows, instruction j covers rows 8 j .. 8 j + 7 (lane: row 8 j + lane / 8,
    // 16-byte chunk (lane & 7) ^ ((row >> 1) & 7): the kimg_off image read by the fp8 fragments)
    static constexpr int NR = SK == PP_SK ? ROWS / 16 : ROWS / 8;
    static constexpr int NI = (NR + 7) / 8;
    const bf16_t* src[NI];
    int dst[NI];
    long step;

    __device__ __forceinline__ void init(const bf16_t* p, long ld, int extent, int base, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            int j = wave * NI + i;
            j = j < NR ? j : NR - 1;
            dst[i] = j * 512;
            if constexpr (KMAJ && SK != PP_SK) {
                const int row = 8 * j + (lane >> 3);
                const int g = min(base + row, extent - 1);
                src[i] = p + (long)g * ld + (((lane & 7) ^ ((row >> 1) & 7)) << 3);
            } else if constexpr (KMAJ) {
                const int row = 16 * j + (lane >> 2);
                const int g = min(base + row, extent - 1);
                src[i] = p + (long)g * ld + (((lane & 3) ^ pp_swz(row)) << 3);
            } else {
                constexpr int CPR = ROWS / 8, RPI = 64 / CPR;
                const int kr = RPI * j + lane / CPR;
                const int c = (lane % CPR) ^ ((mimg_off<ROWS>(kr, 0) - kr * ROWS) >> 3);
                const int col = min(base + 8 * c, extent - 8);
                src[i] = p + (long)kr * ld + col;
            }
        }
        step = KMAJ ? SK : SK * ld;
    }
    __device__ __forceinline__ void skip(int slices) {
#pragma unroll
        for (int i = 0; i < NI; ++i) src[i] += slices * step;
    }
    __device__ __forceinline__ void issue(bf16_t* img, int s) const {
#pragma unroll
        for (int i = 0; i < NI; ++i)
            __builtin_amdgcn_global_load_lds(src[i] + s * step, (lds_void*)(img + dst[i]), 16, 0, 0);
    }
    // copy the next slice and advance (the hot-loop form: one 64-bit add per instruction, no multiply)
    __device__ __forceinline__ void issue_next(bf16_t* img) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            __builtin_amdgcn_global_load_lds(src[i], (lds_void*)(img + dst[i]), 16, 0, 0);
            src[i] += step;
        }
    }
};

template <int N>
__device__ __forceinline__ void pp_vmwait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// retire all but `keep` slices of this wave's copies (keep = slices allowed to stay in flight)
template <int NIT, int DMAX>
__device__ __forceinline__ void pp_retire(int keep) {
    if constexpr (DMAX >= 5) { if (keep >= 5) { pp_vmwait<5 * NIT>(); return; } }
    if constexpr (DMAX >= 4) { if (keep == 4) { pp_vmwait<4 * NIT>(); return; } }
    if constexpr (DMAX >= 3) { if (keep == 3) { pp_vmwait<3 * NIT>(); return; } }
    if constexpr (DMAX >= 2) { if (keep == 2) { pp_vmwait<2 * NIT>(); return; } }
    if (keep == 1) { pp_vmwait<NIT>(); return; }
    if (keep == 0) pp_vmwait<0>();
}

// Persistent over work items (tile, K-split): block b takes items b, b + G, ... (G = gridDim.x, a
// multiple of 8, so an item keeps its block's XCD label).  The K-slices of consecutive items form one
// continuous stream through the ring: the copies of the next item's first slices are in flight while the
// current item finishes and stores its tile, so a tile boundary costs only the epilogue.
// FX (fusions, FX_* bits): A-operand BN-affine+ReLU prologue, BN partial statistics of the output,
// BN-backward masking + statistics (the conv/1x1 paths of the ResNet blocks).
template <class C, int AM, int BMODE, int EM, int FX = 0>
__global__ void __launch_bounds__(512, 2) gemm_pp_kernel(GemmArgs a) {
    constexpr bool AK = AM == A_KMAJOR, BKm = BMODE == B_KMAJOR;
    static_assert(!(FX & FX_PRO) || AK, "prologue: K-major A only");
    constexpr int NB = C::NB, D = NB - 1;
    static_assert(!C::DT || (AK && BKm && (C::DT == 2 || !(FX & FX_PRO))), "fp8 / 64-deep: K-major operands");
    using LA = PPLoader<PP_BM, AK, C::SK>;
    using LB = PPLoader<C::BN, BKm, C::SK>;
    constexpr int NIT = LA::NI + LB::NI;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const sb = reinterpret_cast<bf16_t*>(smem);
    float* const ptab = reinterpret_cast<float*>(smem + C::SMEM);     // FX_PRO: [scale | shift] per k

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if constexpr ((FX & FX_PRO) != 0) {
        for (int i = tid; i < a.K; i += 512) {
            ptab[i] = a.pro_scale[i];
            ptab[PP_PRO_MAXK + i] = a.pro_shift[i];
        }
    }
    if constexpr ((FX & FX_BNB) != 0) {     // the BN-output ReLU mask coefficients of every column
        for (int i = tid; i < a.N; i += 512) {
            ptab[i] = a.ep_mscale[i];
            ptab[PP_PRO_MAXK + i] = a.ep_mshift[i];
        }
    }
    const int grp = wave >> 2, wr = (wave & 3) / C::WC, wc = (wave & 3) % C::WC;
    const int tiles_m = (a.M + PP_BM - 1) / PP_BM, tiles_n = (a.N + C::BN - 1) / C::BN;
    const int ntiles = tiles_m * tiles_n;
    const int splits = a.nb2 > 0 ? a.nb2 : 1;                  // K-splits (slab epilogue when > 1)
    // slices of K-split z: nsl, one more for the first `rem` splits (split z starts at z nsl + min(z, rem))
    const int nsl = a.ktiles_per_split, rem = a.ksl_rem;
    const int G = gridDim.x, b = blockIdx.x;
    const int nitems = (ntiles * splits - b + G - 1) / G;
    if (nitems <= 0 || nsl <= 0) return;                         // uniform over the block
    auto item_nsl = [&](int i) { return nsl + ((b + i * G) / ntiles < rem ? 1 : 0); };
    int Q = nitems * nsl;                                        // slices this block consumes
    if (rem)
        for (int i = 0; i < nitems; ++i) Q += item_nsl(i) - nsl;

    // work item i of this block -> (m0, n0, first slice, split)
    auto item = [&](int i, int& m0, int& n0, int& z) {
        const int w = b + i * G;
        z = w / ntiles;
        const int t = xcd_remap(w - z * ntiles, ntiles);
        const int gsz = PP_GROUP * tiles_n, gid = t / gsz, first = gid * PP_GROUP;
        const int gm = min(tiles_m - first, PP_GROUP), r = t - gid * gsz;
        m0 = (first + r % gm) * PP_BM;
        n0 = (r / gm) * C::BN;
    };

    LA la;
    LB lb;
    // issue cursor (slices run ahead of the compute cursor by up to D): loaders point at the next slice
    int iss_item = 0, iss_s = 0, iss_n = nsl, wr_off = 0;
    auto load_item = [&](int i) {
        int m0, n0, z;
        item(i, m0, n0, z);
        la.init(a.A, a.lda, a.M, m0, wave, lane);
        lb.init(a.B, a.ldb, a.N, n0, wave, lane);
        const int k0 = z * nsl + min(z, rem);
        la.skip(k0);
        lb.skip(k0);
        iss_n = item_nsl(i);
    };
    auto issue_next = [&]() {                                    // copy the next stream slice into its slot
        bf16_t* img = sb + wr_off;
        la.issue_next(img);
        lb.issue_next(img + C::IMA);
        wr_off = wr_off + C::SLOT == NB * C::SLOT ? 0 : wr_off + C::SLOT;
        if (++iss_s == iss_n) {
            iss_s = 0;
            if (++iss_item < nitems) load_item(iss_item);
        }
    };

    f32x4_t acc[C::FM][C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // fused row sums of A (E_F32 with a.rowsum: the bias gradient beside a weight gradient): the waves of the
    // first column block of each n0 == 0 item add one MFMA per A fragment against a ones fragment
    constexpr bool RS = EM == E_F32 && FX == 0 && C::DT == 0;
    f32x4_t accr[RS ? C::FM : 1];
#pragma unroll
    for (int i = 0; i < (RS ? C::FM : 1); ++i) accr[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // optional phase trace: [block][wave 0 / 4][0 start, 1 prologue done, 2 + 2i item i computed, 3 + 2i stored]
    long long* const dbg = (a.dbg && lane == 0 && (wave & 3) == 0) ? a.dbg + ((long)b * 2 + grp) * 64 : nullptr;
    if (dbg) dbg[0] = wall_clock64();
    // prologue: stream slices 0 .. D-1, then retire slice 0
    load_item(0);
    for (int q = 0; q < D && q < Q; ++q) issue_next();
    pp_retire<NIT, D>(min(Q, D) - 1);
    if (dbg) dbg[1] = wall_clock64();
    if constexpr ((FX & (FX_PRO | FX_BNB)) != 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // table written
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();          // stagger: group 1 runs one barrier behind

    const int koffl = pp_koff(lane & 15, lane >> 4);     // K-major fragment offset (row & 15 == lane & 15)
    const int arow = grp * 128 + wr * C::WTM, bcol = wc * C::WTN;
    const int lm = lane & 15, lg = lane >> 4;
    float alpha = a.alpha;
    if (a.alpha_ptr) alpha *= *a.alpha_ptr;
    // output row of GEMM row m: m itself, or with `scatter` the pixel (n, st*y + ph, st*x + pw) of the strided
    // conv's input grid that row m = (n, y, x) of the parity class maps to (the 1x1 stride-2 data gradient)
    auto orow_of = [&](int m) -> long {
        if (!a.scatter) return m;
        const uint32_t nn = fdiv((uint32_t)m, a.g.dHW);
        const uint32_t rem = (uint32_t)m - nn * a.g.dHW.d;
        const uint32_t hc = fdiv(rem, a.g.dW);
        const uint32_t wc = rem - hc * a.g.dW.d;
        return ((long)nn * a.g.H + hc * a.g.st + a.g.ph) * a.g.W + wc * a.g.st + a.g.pw;
    };

    int s = 0, cur = 0, rd_off = 0;                      // slice within the current item, item index, read slot
    int cur_n = item_nsl(0);                             // slices of item `cur`
    // row sums this item: a.rowsum set, the item's first column tile, this wave's first column block
    auto rs_on = [&](int i) {
        if constexpr (!RS) return false;
        int m0_, n0_, z_;
        item(i, m0_, n0_, z_);
        return a.rowsum != nullptr && n0_ == 0 && wc == 0;
    };
    bool cur_rs = rs_on(0);
    // Deferred store drain (tuning pp_epi_slack, plain bf16 epilogues): vmcnt counts stores too on gfx9 and
    // retires in issue order, so the first load wait after an epilogue -- vmcnt((D-2) NIT) for the next slice --
    // also waited for every store of the tile just written.  Here the epilogue stores are buffer stores (lanes
    // past the edges get an offset beyond the range, which the hardware drops), so every wave issues exactly
    // SE0 (SE1 with the GELU pre-activation) of them per item, and the next D-1 load segments, whose awaited
    // slices were issued before those stores, wait for vmcnt((D-2) NIT + SE) instead: the stores drain under
    // the next item's MFMAs.
    // (fp32 epilogues -- weight gradients, split-K slabs -- likewise: one 16-byte store per fragment)
    constexpr bool SLK = (EM == E_BF16 || EM == E_F32) && FX == 0;
    constexpr int SE0 = EM == E_F32 ? C::FM * C::FN : C::FM * (C::FN / 2 + C::FN % 2);
    constexpr int SE1 = EM == E_F32 ? SE0 : SE0 + C::FM * C::FN;
    static_assert(!SLK || (D - 2) * NIT + SE1 <= 63, "vmcnt immediate");
    const bool slk_on = SLK && a.epi_slack > 0;
    const bool slk_aux = slk_on && a.relu == 2 && a.ep_aux != nullptr;
    int slk = 0;                                         // load segments left that may wait with the stores in flight
    constexpr uint32_t OOB = 0x80000000u;                // > any range (epi_slack < 2^31)
    auto epilogue = [&]() {
            // ---------------- epilogue of item `cur`: lane holds C[m0 + arow + 16 fm + lm][n0 + bcol + 16 fn + 4 lg + j]
            if (dbg && cur < 31) dbg[2 + 2 * cur] = wall_clock64();
            s = 0;
            int m0, n0, z;
            const bool rs_here = cur_rs;
            item(cur++, m0, n0, z);
            cur_n = item_nsl(cur);
            cur_rs = cur < nitems && rs_on(cur);
            constexpr bool SUMS = (FX & (FX_STATS | FX_BNB)) != 0;
            float s_[SUMS ? C::FN : 1][4], q_[SUMS ? C::FN : 1][4];   // per-column partial sums over 64 rows
            if constexpr (SUMS) {
#pragma unroll
                for (int fn = 0; fn < C::FN; ++fn)
#pragma unroll
                    for (int j = 0; j < 4; ++j) s_[fn][j] = q_[fn][j] = 0.f;
            }
            // Plain bf16 epilogues: the bias of this lane's columns is loaded once per item, and the residual /
            // dGELU operand one fragment row ahead of its use.  Every load is issued before the stores of the
            // rows after it (s_waitcnt vmcnt counts stores too on gfx9, so a load issued after a store waits for
            // it) and unconditionally, from clamped addresses.  Loading both per fragment inside the row loop
            // serialised ~FM x FN load latencies behind the stores: +13 us for the bias alone on the GPT-2 fc
            // shape (dev/probes/epi_cost.py, gpurun_out/r4_13).
            // (the 288-wide tile keeps the operand loads per fragment: its prefetch registers spilled to scratch;
            // it runs the GPT-2 qkv GEMM, whose epilogue has only a bias)
            // The BN-backward epilogue prefetches its BN input t the same way (the 1x1 conv3 data gradients).
            constexpr bool PF = EM == E_BF16 && FX == 0;
            constexpr bool PFO = (PF || (EM == E_BF16 && FX == FX_BNB)) && C::FN <= 8;
            const bf16_t* const eop = !PFO ? nullptr : FX == FX_BNB ? a.ep_x : (a.ep_dgelu ? a.ep_dgelu : a.ep_res);
            float4 bia[PF ? C::FN : 1];
            u16x4_t nx[PFO ? C::FN : 1];
            auto load_op = [&](int fm_) {      // PFO only
                const long mm = orow_of(min(m0 + arow + fm_ * 16 + lm, a.M - 1));
#pragma unroll
                for (int fn = 0; fn < C::FN; ++fn) {
                    const int n = min(n0 + bcol + fn * 16 + 4 * lg, a.N - 4);
                    nx[fn] = *reinterpret_cast<const u16x4_t*>(eop + mm * a.ldc + n);
                }
            };
            if constexpr (PF) {
#pragma unroll
                for (int fn = 0; fn < C::FN; ++fn) {
                    const int n = min(n0 + bcol + fn * 16 + 4 * lg, a.N - 4);
                    bia[fn] = a.bias ? *reinterpret_cast<const float4*>(a.bias + n) : float4{0.f, 0.f, 0.f, 0.f};
                }
            }
            if constexpr (PFO) {
                if (eop) load_op(0);
            }
            static_for<0, C::FM>([&](auto FMC) {
                constexpr int fm = decltype(FMC)::value;
                // BN-backward epilogue: keep each fragment's loads inside its own iteration (hoisted loads of
                // every fragment's t / coefficients pushed the 256-wide variant into scratch)
                if constexpr ((FX & FX_BNB) != 0) __builtin_amdgcn_sched_barrier(0);
                const int m = m0 + arow + fm * 16 + lm;
                const bool mv = m < a.M;
                const long orow = orow_of(mv ? m : 0);
                if constexpr (EM == E_BF16) {
                    uint32_t pk[C::FN][2];
                    u16x4_t cu[PFO ? C::FN : 1];
                    if constexpr (PFO) {
                        if (eop) {
#pragma unroll
                            for (int fn = 0; fn < C::FN; ++fn) cu[fn] = nx[fn];
                            if constexpr (fm + 1 < C::FM) load_op(fm + 1);
                        }
                    }
#pragma unroll
                    for (int fn = 0; fn < C::FN; ++fn) {
                        const int n = n0 + bcol + fn * 16 + 4 * lg;
                        const bool ok = mv && n + 4 <= a.N;
                        const long off = orow * a.ldc + n;
                        float v[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = acc[fm][fn][j] * alpha;
                        if constexpr (PF) {
                            if (a.bias) {
                                v[0] += bia[fn].x; v[1] += bia[fn].y; v[2] += bia[fn].z; v[3] += bia[fn].w;
                            }
                        } else if (a.bias && n + 4 <= a.N) {
                            const float4 bb = *reinterpret_cast<const float4*>(a.bias + n);
                            v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
                        }
                        if (a.relu == 1) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
                        } else if (a.relu == 2) {
                            u16x4_t pre;
#pragma unroll
                            for (int j = 0; j < 4; ++j) pre[j] = f2bf(v[j]);
                            if (slk_aux) {
                                const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
                                    a.ep_aux, 0, a.epi_slack, 0x00020000);
                                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, pre), xr,
                                                                      ok ? (uint32_t)(off * 2) : OOB, 0, 0);
                            } else if (a.ep_aux && ok) {
                                *reinterpret_cast<u16x4_t*>(a.ep_aux + off) = pre;
                            }
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(bf2f(pre[j]));
                        }
                        if (a.ep_dgelu && ok) {
                            u16x4_t u;
                            if constexpr (PFO && FX == 0) u = cu[fn];
                            else u = *reinterpret_cast<const u16x4_t*>(a.ep_dgelu + off);
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] *= gelu_tanh_grad(bf2f(u[j]));
                        }
                        if (a.ep_res && ok) {
                            u16x4_t r;
                            if constexpr (PFO && FX == 0) r = a.ep_dgelu ? *reinterpret_cast<const u16x4_t*>(a.ep_res + off) : cu[fn];
                            else r = *reinterpret_cast<const u16x4_t*>(a.ep_res + off);
                            const uint32_t mb = a.ep_rmask ? (uint32_t)(a.ep_rmask[off >> 3] >> (off & 4)) : 0xFu;
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] += ((mb >> j) & 1) ? bf2f(r[j]) : 0.f;
                        }
                        if constexpr ((FX & FX_BNB) != 0) {
                            // gm = v * [t*mscale + mshift > 0] (ReLU mask of the BN output recomputed from its
                            // input t); sums of gm and gm * t here, sum gm * xhat = invstd (sum gm t - mean sum gm)
                            // at the flush (per-fragment mean / invstd loads pushed this variant into scratch)
                            u16x4_t tv = {0, 0, 0, 0};
                            float4 ms = {0, 0, 0, 0}, mh = ms;
                            if constexpr (PFO) tv = cu[fn];          // (masked by `ok` below)
                            else if (ok) tv = *reinterpret_cast<const u16x4_t*>(a.ep_x + off);
                            ms = *reinterpret_cast<const float4*>(ptab + n);
                            mh = *reinterpret_cast<const float4*>(ptab + PP_PRO_MAXK + n);
                            const float msa[4] = {ms.x, ms.y, ms.z, ms.w}, mha[4] = {mh.x, mh.y, mh.z, mh.w};
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const float tt = bf2f(tv[j]);
                                const float gm = (ok && fmaf(tt, msa[j], mha[j]) > 0.f) ? bf2f(f2bf(v[j])) : 0.f;
                                v[j] = gm;
                                s_[fn][j] += gm;
                                q_[fn][j] += gm * tt;
                            }
                        } else if constexpr ((FX & FX_STATS) != 0) {
                            if (ok) {
#pragma unroll
                                for (int j = 0; j < 4; ++j) {
                                    const float rr = bf2f(f2bf(v[j]));
                                    s_[fn][j] += rr;
                                    q_[fn][j] += rr * rr;
                                }
                            }
                        }
                        pk[fn][0] = pk2bf(v[0], v[1]);
                        pk[fn][1] = pk2bf(v[2], v[3]);
                    }
                    bf16_t* const Crow = reinterpret_cast<bf16_t*>(a.C) + orow * a.ldc;
                    [[maybe_unused]] __amdgpu_buffer_rsrc_t cr;
                    if constexpr (SLK) cr = __builtin_amdgcn_make_buffer_rsrc(a.C, 0, a.epi_slack, 0x00020000);
#pragma unroll
                    for (int fp = 0; fp < C::FN / 2; ++fp) {   // 16-byte stores: permlane16 swap pairs fragments
                        const auto s0_ = __builtin_amdgcn_permlane16_swap(pk[2 * fp][0], pk[2 * fp + 1][0], false, false);
                        const auto s1_ = __builtin_amdgcn_permlane16_swap(pk[2 * fp][1], pk[2 * fp + 1][1], false, false);
                        const int n = n0 + bcol + (2 * fp + (lg & 1)) * 16 + 8 * (lg >> 1);
                        if (slk_on) {                          // (N % 8 == 0: whole 16-byte groups)
                            const uint32_t bo = mv && n + 8 <= a.N ? (uint32_t)((orow * a.ldc + n) * 2) : OOB;
                            __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{s0_[0], s1_[0], s0_[1], s1_[1]}, cr, bo, 0, 0);
                        } else if (mv && n + 8 <= a.N) {
                            *reinterpret_cast<uint4*>(Crow + n) = make_uint4(s0_[0], s1_[0], s0_[1], s1_[1]);
                        } else if (mv && n < a.N) {
                            const uint32_t w4[4] = {s0_[0], s1_[0], s0_[1], s1_[1]};
                            for (int j = 0; j < 8 && n + j < a.N; ++j) Crow[n + j] = (bf16_t)(w4[j >> 1] >> (16 * (j & 1)));
                        }
                    }
                    if constexpr (C::FN % 2) {                 // odd fragment count: 8-byte stores for the last one
                        const int n = n0 + bcol + (C::FN - 1) * 16 + 4 * lg;
                        if (slk_on) {
                            const uint32_t bo = mv && n + 4 <= a.N ? (uint32_t)((orow * a.ldc + n) * 2) : OOB;
                            __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{pk[C::FN - 1][0], pk[C::FN - 1][1]}, cr, bo, 0, 0);
                        } else if (mv && n + 4 <= a.N) {
                            *reinterpret_cast<uint2*>(Crow + n) = make_uint2(pk[C::FN - 1][0], pk[C::FN - 1][1]);
                        }
                    }
                    if constexpr (SUMS) {
                        // flush one slab row pair per 64 rows (4 fragments) of the wave; the slab has one row pair
                        // per 64 rows of M rounded up to 128 (the layout of the 128-row kernel)
                        if constexpr (fm % 4 == 3 || fm == C::FM - 1) {
#pragma unroll
                            for (int fn = 0; fn < C::FN; ++fn)
#pragma unroll
                                for (int j = 0; j < 4; ++j) {
                                    s_[fn][j] = row16_sum(s_[fn][j]);
                                    q_[fn][j] = row16_sum(q_[fn][j]);
                                }
                            const int g64 = m0 + arow + (fm / 4) * 64;
                            if (g64 < ((a.M + 127) / 128) * 128) {
#pragma unroll
                                for (int fn = 0; fn < C::FN; ++fn) {
                                    const int n = n0 + bcol + fn * 16 + 4 * lg;
                                    const int jj = lm & 3;
                                    const bool okn = n + jj < a.N;
                                    if constexpr ((FX & FX_BNB) != 0) {
                                        // lanes lm 4..7 add column jj's sum gm * xhat (their own mean / invstd)
                                        if ((lm & 12) == 4 && okn) {
                                            const float qj = a.ep_invstd[n + jj] *
                                                             (sel4(q_[fn], jj) - a.ep_mean[n + jj] * sel4(s_[fn], jj));
                                            q_[fn][0] = q_[fn][1] = q_[fn][2] = q_[fn][3] = qj;
                                        }
                                    }
                                    float* ps = stat_row(a.stats, g64 / 64, a.N) + n;
                                    stat_add_frag(ps, ps + a.N, lane, s_[fn], q_[fn], okn);
                                }
                            }
#pragma unroll
                            for (int fn = 0; fn < C::FN; ++fn)
#pragma unroll
                                for (int j = 0; j < 4; ++j) s_[fn][j] = q_[fn][j] = 0.f;
                        }
                    }
                } else {
                    if constexpr (RS) {
                        // lane (lm, lg): every column of accr[fm] holds row m's sum; lanes of column group 0 add it
                        if (rs_here && lg == 0 && mv) atomicAdd(a.rowsum + m, accr[fm][0] * alpha);
                        accr[fm] = f32x4_t{0.f, 0.f, 0.f, 0.f};
                    }
                    // fp32: K-split items write partial slabs at C + z * sC1 (pp_slab_reduce_kernel sums them),
                    // otherwise store / accumulate (acc_c) into C
                    const bool slab = splits > 1;
                    float* const Cb = reinterpret_cast<float*>(a.C) + (slab ? z * a.sC1 : 0);
                    [[maybe_unused]] __amdgpu_buffer_rsrc_t cr;
                    if constexpr (SLK) cr = __builtin_amdgcn_make_buffer_rsrc(Cb, 0, a.epi_slack, 0x00020000);
#pragma unroll
                    for (int fn = 0; fn < C::FN; ++fn) {
                        const int n = n0 + bcol + fn * 16 + 4 * lg;
                        if (slk_on) {              // (N, ldc % 4 == 0: whole float4 groups; no bias / activation)
                            const bool ok = mv && n < a.N;
                            float v[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = acc[fm][fn][j] * alpha;
                            if (a.acc_c && !slab && ok) {
                                const float4 o = *reinterpret_cast<const float4*>(Cb + (long)m * a.ldc + n);
                                v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
                            }
                            __builtin_amdgcn_raw_buffer_store_b128(
                                __builtin_bit_cast(u32x4_t, f32x4_t{v[0], v[1], v[2], v[3]}), cr,
                                ok ? (uint32_t)(((long)m * a.ldc + n) * 4) : OOB, 0, 0);
                            continue;
                        }
                        if (!mv || n >= a.N) continue;
                        float v[4];
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = acc[fm][fn][j] * alpha;
                        float* Cp = Cb + (long)m * a.ldc + n;
                        const bool n4 = n + 4 <= a.N;
                        if (!slab && a.bias && n4) {
                            const float4 bb = *reinterpret_cast<const float4*>(a.bias + n);
                            v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
                        }
                        if (!slab && a.relu == 1) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
                        } else if (!slab && a.relu == 2) {
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(v[j]);
                        }
                        if (n4 && (a.ldc & 3) == 0) {
                            float4* C4 = reinterpret_cast<float4*>(Cp);
                            if (a.acc_c && !slab) {
                                const float4 o = *C4;
                                v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
                            }
                            *C4 = make_float4(v[0], v[1], v[2], v[3]);
                        } else {
                            for (int j = 0; j < 4 && n + j < a.N; ++j) Cp[j] = v[j] + ((a.acc_c && !slab) ? Cp[j] : 0.f);
                        }
                    }
                }
            });
            if (dbg && cur <= 31) dbg[1 + 2 * cur] = wall_clock64();
#pragma unroll
            for (int i = 0; i < C::FM; ++i)
#pragma unroll
                for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            if (slk_on) slk = D - 1;
    };
    {
        for (int q = 0; q < Q; ++q) {
            // ---------------- load segment ----------------
            const bool more = q + D < Q;
            if (more) {                                  // stream slice q+1 landed (this wave's copies)
                if constexpr (SLK) {
                    if (slk > 0) {                       // ... issued before the last epilogue's stores
                        --slk;
                        if (slk_aux) pp_vmwait<(D - 2) * NIT + SE1>();
                        else pp_vmwait<(D - 2) * NIT + SE0>();
                    } else {
                        pp_vmwait<(D - 2) * NIT>();
                    }
                } else {
                    pp_vmwait<(D - 2) * NIT>();
                }
            } else {
                pp_retire<NIT, D>(Q - q - 2);
            }
            const bf16_t* A_ = sb + rd_off;
            const bf16_t* B_ = A_ + C::IMA;
            rd_off = rd_off + C::SLOT == NB * C::SLOT ? 0 : rd_off + C::SLOT;
            bf16x8_t af[C::DT ? 1 : C::FM], bfr[C::DT ? 1 : C::FN];
            v8i_t aq[C::DT == 1 ? C::FM : 1], bq[C::DT == 1 ? C::FN : 1];   // fp8: 32 k-bytes per lane and fragment
            bf16x8_t a2[C::DT == 2 ? 2 : 1][C::DT == 2 ? C::FM : 1], b2[C::DT == 2 ? 2 : 1][C::DT == 2 ? C::FN : 1];
            if constexpr (C::DT == 2) {      // bf16, 64-deep slices: two 32-deep k-steps per 128-byte row
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
                    for (int f = 0; f < C::FN; ++f) b2[ks][f] = frag_kmajor(B_, bcol + f * 16 + (lane & 15), ks, lane);
#pragma unroll
                    for (int f = 0; f < C::FM; ++f) a2[ks][f] = frag_kmajor(A_, arow + f * 16 + (lane & 15), ks, lane);
                }
            } else if constexpr (C::DT == 1) {
#pragma unroll
                for (int f = 0; f < C::FN; ++f) bq[f] = frag8(B_, bcol + f * 16 + (lane & 15), lane);
#pragma unroll
                for (int f = 0; f < C::FM; ++f) aq[f] = frag8(A_, arow + f * 16 + (lane & 15), lane);
            } else {
#pragma unroll
            for (int f = 0; f < C::FN; ++f) {
                if constexpr (BKm) bfr[f] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(
                                               B_ + (bcol + f * 16) * PP_SK + koffl));
                else bfr[f] = frag_mnmajor<C::BN>(B_, bcol + f * 16, 0, lane);
            }
#pragma unroll
            for (int f = 0; f < C::FM; ++f) {
                if constexpr (AK) af[f] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(
                                              A_ + (arow + f * 16) * PP_SK + koffl));
                else af[f] = frag_mnmajor<PP_BM>(A_, arow + f * 16, 0, lane);
            }
            }
            if (more) issue_next();
            if constexpr ((FX & FX_PRO) != 0 && C::DT == 2) {
                // 64-deep slice: k-step ks of this lane covers k = 64 s + 32 ks + 8 lg .. +7
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const float* ps = ptab + s * 64 + ks * 32 + 8 * (lane >> 4);
                    const float4 c0 = *reinterpret_cast<const float4*>(ps), c1 = *reinterpret_cast<const float4*>(ps + 4);
                    const float4 h0 = *reinterpret_cast<const float4*>(ps + PP_PRO_MAXK);
                    const float4 h1 = *reinterpret_cast<const float4*>(ps + PP_PRO_MAXK + 4);
                    const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
                    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
                    for (int f = 0; f < C::FM; ++f) {
                        u16x8_t v = __builtin_bit_cast(u16x8_t, a2[ks][f]);
#pragma unroll
                        for (int j = 0; j < 8; ++j) v[j] = f2bf(fmaxf(fmaf(bf2f(v[j]), sc[j], sh[j]), 0.f));
                        a2[ks][f] = __builtin_bit_cast(bf16x8_t, v);
                    }
                }
            } else if constexpr ((FX & FX_PRO) != 0) {
                // this lane's 8 reduction indices of the slice: k = 32 s + 8 lg .. +7 (no split-K with FX_PRO)
                const float* ps = ptab + s * PP_SK + 8 * (lane >> 4);
                const float4 c0 = *reinterpret_cast<const float4*>(ps), c1 = *reinterpret_cast<const float4*>(ps + 4);
                const float4 h0 = *reinterpret_cast<const float4*>(ps + PP_PRO_MAXK);
                const float4 h1 = *reinterpret_cast<const float4*>(ps + PP_PRO_MAXK + 4);
                const float sc[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
                const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
                for (int f = 0; f < C::FM; ++f) {
                    u16x8_t v = __builtin_bit_cast(u16x8_t, af[f]);
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = f2bf(fmaxf(fmaf(bf2f(v[j]), sc[j], sh[j]), 0.f));
                    af[f] = __builtin_bit_cast(bf16x8_t, v);
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            // ---------------- compute segment ----------------
            __builtin_amdgcn_s_setprio(1);
            if constexpr (C::DT == 2) {
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
                        for (int fn = 0; fn < C::FN; ++fn)
                            acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2[ks][fn], a2[ks][fm], acc[fm][fn], 0, 0, 0);
            } else if constexpr (C::DT == 1) {
#pragma unroll
                for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
                    for (int fn = 0; fn < C::FN; ++fn)
                        acc[fm][fn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                            bq[fn], aq[fm], acc[fm][fn], 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
            } else {
#pragma unroll
            for (int fm = 0; fm < C::FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < C::FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af[fm], acc[fm][fn], 0, 0, 0);
            if constexpr (RS) {
                if (cur_rs) {
                    const bf16x8_t ones = __builtin_bit_cast(bf16x8_t, u16x8_t{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80,
                                                                              0x3F80, 0x3F80, 0x3F80});
#pragma unroll
                    for (int fm = 0; fm < C::FM; ++fm)
                        accr[fm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, af[fm], accr[fm], 0, 0, 0);
                }
            }
            }
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            if (++s < cur_n) continue;
            // epilogue pairing (tuning pp_epi_pair): the staggered groups would write their halves of the tile in
            // consecutive barrier intervals, each one's epilogue beside the other's last / first compute segment,
            // i.e. two epilogue-long intervals per item with one wave per SIMD working.  Group 0 waits out group
            // 1's last compute segment at one extra barrier and group 1 takes one extra barrier after its
            // epilogue: both epilogues share one interval and the stagger resumes (RAW / WAR of the ring unchanged:
            // every read and refill keeps its order against the barriers it depended on)
            if (a.epi_pair && grp == 0) __builtin_amdgcn_s_barrier();
            epilogue();
            if (a.epi_pair && grp == 1) __builtin_amdgcn_s_barrier();
        }
        if (grp == 0) __builtin_amdgcn_s_barrier();      // balance the stagger
    }
}

// out[m][n] (+)= sum_z slab[z][m][n]  (fp32, ld = ldc, slab stride sz).  float4 per thread.
// s += slab rows z, z + ST, ... (< splits) for the < 8 rows left after an 8-wide loop: 4 / 2 / 1 loads at a time
template <int ST>
__device__ __forceinline__ void pp_sum_tail(const float* __restrict__ slab, long sz, long soff, int z, int splits,
                                            float4& s) {
    if (z + 3 * ST < splits) {
        float4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = *reinterpret_cast<const float4*>(slab + (z + ST * j) * sz + soff);
#pragma unroll
        for (int j = 0; j < 4; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
        z += 4 * ST;
    }
    if (z + ST < splits) {
        const float4 v0 = *reinterpret_cast<const float4*>(slab + z * sz + soff);
        const float4 v1 = *reinterpret_cast<const float4*>(slab + (z + ST) * sz + soff);
        s.x += v0.x + v1.x; s.y += v0.y + v1.y; s.z += v0.z + v1.z; s.w += v0.w + v1.w;
        z += 2 * ST;
    }
    if (z < splits) {
        const float4 v = *reinterpret_cast<const float4*>(slab + z * sz + soff);
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
}

__global__ void __launch_bounds__(256) pp_slab_reduce_kernel(const float* __restrict__ slab, long sz, int splits,
                                                             float* __restrict__ out, int M, int N, long ldc,
                                                             int accumulate) {
    const int n4 = N >> 2;
    const long total = (long)M * n4;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int m = (int)(i / n4), c = (int)(i - (long)m * n4) * 4;
        const long off = (long)m * ldc + c, soff = (long)m * N + c;       // slab rows are N wide
        float4 s = accumulate ? *reinterpret_cast<const float4*>(out + off) : make_float4(0.f, 0.f, 0.f, 0.f);
        int z = 0;
        for (; z + 8 <= splits; z += 8) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float4*>(slab + (z + j) * sz + soff);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
        }
        // the remaining < 8 splits as 4 / 2 / 1 loads issued together (a 1-load loop serialised their latencies)
        pp_sum_tail<1>(slab, sz, soff, z, splits, s);
        *reinterpret_cast<float4*>(out + off) = s;
    }
}

__global__ void __launch_bounds__(256) pp_slab_reduce_wide_kernel(const float* __restrict__ slab, long sz, int splits,
                                                             float* __restrict__ out, int M, int N, long ldc,
                                                             int accumulate) {
    // a block covers 32 consecutive float4 outputs with 8 split groups: thread (o, zg) sums splits zg, zg + 8, ...
    // (8 loads in flight), the groups are combined through LDS.  One thread per output summing every split was
    // a splits/8-deep latency chain on a grid of only M*N/1024 blocks (31-49 us per 1x1 conv weight gradient).
    __shared__ float4 red[8][32];
    const int o = threadIdx.x & 31, zg = threadIdx.x >> 5;
    const int n4 = N >> 2;
    const long total = (long)M * n4;
    const long i = (long)blockIdx.x * 32 + o;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    long off = 0;
    if (i < total) {
        const int m = (int)(i / n4), c = (int)(i - (long)m * n4) * 4;
        off = (long)m * ldc + c;
        const long soff = (long)m * N + c;        // slab rows are N wide
        int z = zg;
        for (; z + 56 < splits; z += 64) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float4*>(slab + (z + 8 * j) * sz + soff);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
        }
        pp_sum_tail<8>(slab, sz, soff, z, splits, s);
    }
    red[zg][o] = s;
    __syncthreads();
    if (zg == 0 && i < total) {
#pragma unroll
        for (int k = 1; k < 8; ++k) { const float4 v = red[k][o]; s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
        if (accumulate) {
            const float4 cur = *reinterpret_cast<const float4*>(out + off);
            s.x += cur.x; s.y += cur.y; s.z += cur.z; s.w += cur.w;
        }
        *reinterpret_cast<float4*>(out + off) = s;
    }
}

// out_bf16[m][n] = bf16(sum_z slab[z][m][n])
__global__ void __launch_bounds__(256) pp_slab_reduce_bf16_kernel(const float* __restrict__ slab, long sz, int splits,
                                                                  bf16_t* __restrict__ out, int M, int N, long ldc) {
    const int n4 = N >> 2;
    const long total = (long)M * n4;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const int m = (int)(i / n4), c = (int)(i - (long)m * n4) * 4;
        const long off = (long)m * N + c;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        int z = 0;
        for (; z + 8 <= splits; z += 8) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float4*>(slab + (z + j) * sz + off);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
        }
        for (; z < splits; ++z) {
            const float4 v = *reinterpret_cast<const float4*>(slab + z * sz + off);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        u16x4_t o = {f2bf(s.x), f2bf(s.y), f2bf(s.z), f2bf(s.w)};
        *reinterpret_cast<u16x4_t*>(out + (long)m * ldc + c) = o;
    }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
using C96 = PPC<96, 2, 7>;
using C96k = PPC<96, 2, 3, 2>;       // 64-deep bf16 slices: 45 KiB slots, 3 in the ring
using C128k = PPC<128, 2, 3, 2>;     // 48 KiB slots
using C128 = PPC<128, 2, 5>;
using C192 = PPC<192, 2, 5>;
using C256 = PPC<256, 1, 4>;
using C288 = PPC<288, 2, 4>;
using C256b = PPC<256, 1, 5>;        // 160 KiB ring (A/B: PDNN_PP_BN=257)
using C8_128 = PPC<128, 2, 3, 1>;    // fp8: 48 KiB slots (128-byte rows), 3 in the ring
using C8_96 = PPC<96, 2, 3, 1>;

long long* g_pp_trace = nullptr;

// CUs a persistent grid fills (all of them unless RCCL channels are reserved: tuning.h comm_cus)
int device_cus() { return grid_cus(); }


template <class C, int FX>
constexpr int pp_smem() { return C::SMEM + ((FX & (FX_PRO | FX_BNB)) ? 2 * PP_PRO_MAXK * 4 : 0); }

template <class C, int AM, int BMODE, int EM, int FX = 0>
void set_attr() {
    static bool attr = false;
    if (!attr) {
        attr = true;
        static_assert(pp_smem<C, FX>() <= 160 * 1024, "LDS");
        (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<C, AM, BMODE, EM, FX>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, pp_smem<C, FX>());
    }
}

template <class C, int AM, int BMODE, int EM, int FX = 0>
int launch_cfg(const GemmArgs& a, int splits, hipStream_t st) {
    const long items = cdiv(a.M, PP_BM) * cdiv(a.N, C::BN) * splits;
    const int cus = device_cus();
    const int grid = items <= cus ? (int)items : (cus / 8) * 8;     // persistent: one block per CU
    GemmArgs b = a;
    b.nb2 = splits;
    b.dbg = g_pp_trace;
    b.epi_slack = 0;
    b.epi_pair = tune().pp_epi_pair;
    if constexpr (EM == E_BF16 && FX == 0) {
        const long bytes = (long)a.M * a.ldc * 2;
        if (tune().pp_epi_slack && !a.scatter && a.N % 8 == 0 && bytes < (1L << 31)) b.epi_slack = (int)bytes;
    }
    if constexpr (EM == E_F32 && FX == 0) {          // range of one output (or one split-K slab)
        const long bytes = (long)a.M * a.ldc * 4;
        if (tune().pp_epi_slack >= 2 && a.N % 4 == 0 && a.ldc % 4 == 0 && !a.bias && a.relu == 0 && bytes < (1L << 31))
            b.epi_slack = (int)bytes;
    }
    if constexpr (C::DT == 2) {            // 64-deep slices (callers: K % 64 == 0, no split-K)
        b.ktiles_per_split = a.K / 64;
        b.ksl_rem = 0;
    }
    constexpr int SM = pp_smem<C, FX>();
    set_attr<C, AM, BMODE, EM, FX>();
    hipLaunchKernelGGL((gemm_pp_kernel<C, AM, BMODE, EM, FX>), dim3(grid), dim3(512), SM, st, b);
    PDNN_LAUNCH_RET;
}

template <int AM, int BMODE, int EM, int FX = 0>
int launch_bn(const GemmArgs& a, int bn, int splits, hipStream_t st) {
    if constexpr (AM == A_KMAJOR && BMODE == B_KMAJOR && FX == 0) {
        switch (bn) {
            case 96:
                if (tune().pp_sk64 && splits == 1 && a.K % 64 == 0) return launch_cfg<C96k, AM, BMODE, EM>(a, splits, st);
                return launch_cfg<C96, AM, BMODE, EM>(a, splits, st);
            case 128:
                if (tune().pp_sk64 && splits == 1 && a.K % 64 == 0) return launch_cfg<C128k, AM, BMODE, EM>(a, splits, st);
                break;
            case 192: return launch_cfg<C192, AM, BMODE, EM>(a, splits, st);
            case 288: return launch_cfg<C288, AM, BMODE, EM>(a, splits, st);
            case 257: return launch_cfg<C256b, AM, BMODE, EM>(a, splits, st);
            default: break;
        }
    }
    if constexpr (AM == A_KMAJOR && BMODE == B_KMAJOR && EM == E_BF16 && FX != 0) {
        if (bn == 128 && tune().pp_sk64 && splits == 1 && a.K % 64 == 0) return launch_cfg<C128k, AM, BMODE, EM, FX>(a, splits, st);
    }
    if (bn == 128) return launch_cfg<C128, AM, BMODE, EM, FX>(a, splits, st);
    if constexpr ((FX & (FX_BNB | FX_PRO)) == 0) return launch_cfg<C256, AM, BMODE, EM, FX>(a, splits, st);
    return (int)hipErrorInvalidValue;
}

// relative per-CU throughput of the tile widths (A/B measured, tools/pp_check.py)
double bn_eff(int bn) {
    switch (bn) {
        case 96: return 0.78;
        case 128: return 0.86;
        case 192: return 0.93;
        default: return 1.0;
    }
}

// kk: both operands K-major (every tile width); otherwise / with fusions only 128 and 256.
// amn: A (and B) MN-major, the weight-gradient form: both operands are read with ds_read_b64_tr_b16, where the
// 128-wide tile reaches only ~0.65 of the 256-wide one's per-CU rate (GPT-2 LM-head weight gradient
// 50304 x 768 x 8192: 3.1 vs 4.8 TF/s per CU, 934 vs 744 us; gpurun_out/r5_31)
int pick_bn(const GemmArgs& a, bool kk, bool amn = false) {
    const int g_pp_force_bn = tune().pp_bn;
    const int cus = device_cus();
    static const int kk_opts[] = {256, 288, 192, 128, 96};
    static const int mn_opts[] = {256, 128};
    const int* opts = kk ? kk_opts : mn_opts;
    const int nopt = kk ? 5 : 2;
    if (g_pp_force_bn > 0) {
        if (kk && g_pp_force_bn == 257) return 257;
        for (int i = 0; i < nopt; ++i)
            if (opts[i] == g_pp_force_bn) return g_pp_force_bn;
    }
    int best = 256;
    double bt = 1e300;
    for (int i = 0; i < nopt; ++i) {
        const int bn = opts[i];
        const long tiles = cdiv(a.M, PP_BM) * cdiv(a.N, bn);
        const long rounds = cdiv(tiles, cus);
        const double t = (double)rounds * bn / (amn && bn == 128 ? 0.65 : bn_eff(bn));
        if (t < bt * 0.999) { bt = t; best = bn; }
    }
    return best;
}

int fx_of(const GemmArgs& a) {
    return (a.pro_scale ? FX_PRO : 0) | (a.ep_x ? FX_BNB : (a.stats ? FX_STATS : 0));
}

}  // namespace

int& pp_mode_ref() { return tune().pp; }

bool pp_supported(const GemmArgs& a, int amode, int bmode, int em, int batch, int splits) {
    const int mode = pp_mode_ref();
    if (!mode || batch != 1 || splits != 1 || em == E_ATOMIC) return false;
    if (a.causal || a.transC || a.stats_row0) return false;
    if (a.scatter && (em != E_BF16 || fx_of(a) != 0)) return false;      // scatter rows: plain bf16 epilogues
    if (a.K % PP_SK || a.M < 16 || a.N < 16 || a.N % 8 || a.lda % 8 || a.ldb % 8) return false;
    if (!((amode == A_KMAJOR && (bmode == B_KMAJOR || bmode == B_MNMAJOR)) ||
          (amode == A_MNMAJOR && bmode == B_MNMAJOR)))
        return false;
    if (amode == A_MNMAJOR && a.M % 8) return false;
    const int fx = fx_of(a);
    if (fx && em != E_BF16) return false;
    if ((fx & FX_PRO) && (amode != A_KMAJOR || a.K > PP_PRO_MAXK)) return false;
    if ((fx & FX_BNB) && (!a.stats || a.N > PP_PRO_MAXK)) return false;
    if (mode == 2) return true;
    return cdiv(a.M, PP_BM) * cdiv(a.N, 256) >= 48 || (long)a.M * a.N >= (1L << 22);
}

template <int FX>
int pp_launch_fx(const GemmArgs& a, int amode, int bmode, int em, hipStream_t st) {
    // the BN-backward epilogue and the operand prologue fit the 256-wide tile's registers only with scratch
    // spills: 128 wide
    const int bn = (FX & (FX_BNB | FX_PRO)) ? 128
                 : pick_bn(a, FX == 0 && amode == A_KMAJOR && bmode == B_KMAJOR, amode == A_MNMAJOR);
    const int key = amode * 100 + bmode * 10 + em;
    if constexpr (FX != 0) {      // fusions: bf16 output, A K-major
        switch (key) {
            case 0: return launch_bn<A_KMAJOR, B_KMAJOR, E_BF16, FX>(a, bn, 1, st);
            case 10: return launch_bn<A_KMAJOR, B_MNMAJOR, E_BF16, FX>(a, bn, 1, st);
            default: return (int)hipErrorInvalidValue;
        }
    } else {
        switch (key) {
            case 0: return launch_bn<A_KMAJOR, B_KMAJOR, E_BF16>(a, bn, 1, st);
            case 1: return launch_bn<A_KMAJOR, B_KMAJOR, E_F32>(a, bn, 1, st);
            case 10: return launch_bn<A_KMAJOR, B_MNMAJOR, E_BF16>(a, bn, 1, st);
            case 11: return launch_bn<A_KMAJOR, B_MNMAJOR, E_F32>(a, bn, 1, st);
            case 110: return launch_bn<A_MNMAJOR, B_MNMAJOR, E_BF16>(a, bn, 1, st);
            case 111: return launch_bn<A_MNMAJOR, B_MNMAJOR, E_F32>(a, bn, 1, st);
            default: return (int)hipErrorInvalidValue;
        }
    }
}

// fp8 GEMM (both operands K-major e4m3, K / ld in units of 2 bytes, K % 64 units): tile width 128 or 96,
// whichever fills the CUs in fewer rounds (same efficiency weights as the bf16 widths)
int pp_fp8_launch(const GemmArgs& a0, int em, hipStream_t st) {
    GemmArgs a = a0;
    if (a.K % 64 || a.N % 8 || a.M < 16 || a.lda % 8 || a.ldb % 8) return (int)hipErrorInvalidValue;
    a.ktiles_per_split = a.K / 64;
    const int cus = device_cus();
    const double t128 = (double)cdiv(cdiv(a.M, PP_BM) * cdiv(a.N, 128), cus) * 128 / bn_eff(128);
    const double t96 = (double)cdiv(cdiv(a.M, PP_BM) * cdiv(a.N, 96), cus) * 96 / bn_eff(96);
    const bool w96 = tune().pp_bn == 96 || (tune().pp_bn != 128 && t96 < t128 * 0.999);
    if (em == E_F32) return w96 ? launch_cfg<C8_96, A_KMAJOR, B_KMAJOR, E_F32>(a, 1, st)
                                : launch_cfg<C8_128, A_KMAJOR, B_KMAJOR, E_F32>(a, 1, st);
    if (a.stats) return w96 ? launch_cfg<C8_96, A_KMAJOR, B_KMAJOR, E_BF16, FX_STATS>(a, 1, st)
                            : launch_cfg<C8_128, A_KMAJOR, B_KMAJOR, E_BF16, FX_STATS>(a, 1, st);
    return w96 ? launch_cfg<C8_96, A_KMAJOR, B_KMAJOR, E_BF16>(a, 1, st)
               : launch_cfg<C8_128, A_KMAJOR, B_KMAJOR, E_BF16>(a, 1, st);
}

int pp_launch(const GemmArgs& a0, int amode, int bmode, int em, hipStream_t st) {
    GemmArgs a = a0;
    a.ktiles_per_split = a.K / PP_SK;
    switch (fx_of(a)) {
        case 0: return pp_launch_fx<0>(a, amode, bmode, em, st);
        case FX_STATS: return pp_launch_fx<FX_STATS>(a, amode, bmode, em, st);
        case FX_BNB: return pp_launch_fx<FX_BNB>(a, amode, bmode, em, st);
        case FX_PRO: return pp_launch_fx<FX_PRO>(a, amode, bmode, em, st);
        case FX_PRO | FX_STATS: return pp_launch_fx<FX_PRO | FX_STATS>(a, amode, bmode, em, st);
        default: return (int)hipErrorInvalidValue;
    }
}

}  // namespace pg

// hipcc (ROCm 7.2) emits the host launch stub of only the first implicitly instantiated specialisation of
// a kernel template in an anonymous namespace: instantiate every specialisation used explicitly.
#define PP_I(CFG, AM, BM_, EM) template __global__ void pg::gemm_pp_kernel<pg::CFG, pg::AM, pg::BM_, pg::EM, 0>(pg::GemmArgs);
#define PP_I2(CFG, AM, BM_) PP_I(CFG, AM, BM_, E_BF16) PP_I(CFG, AM, BM_, E_F32)
PP_I2(C96, A_KMAJOR, B_KMAJOR) PP_I2(C192, A_KMAJOR, B_KMAJOR)
PP_I2(C96k, A_KMAJOR, B_KMAJOR) PP_I2(C128k, A_KMAJOR, B_KMAJOR) PP_I2(C288, A_KMAJOR, B_KMAJOR)
PP_I2(C128, A_KMAJOR, B_KMAJOR) PP_I2(C256, A_KMAJOR, B_KMAJOR) PP_I2(C256b, A_KMAJOR, B_KMAJOR)
PP_I2(C128, A_KMAJOR, B_MNMAJOR) PP_I2(C256, A_KMAJOR, B_MNMAJOR)
PP_I2(C128, A_MNMAJOR, B_MNMAJOR) PP_I2(C256, A_MNMAJOR, B_MNMAJOR)
#undef PP_I2
#define PP_F(CFG, BM_, FX) template __global__ void pg::gemm_pp_kernel<pg::CFG, pg::A_KMAJOR, pg::BM_, pg::E_BF16, FX>(pg::GemmArgs);
#define PP_F2(BM_, FX) PP_F(C128, BM_, FX) PP_F(C256, BM_, FX)
#define PP_F5(BM_) PP_F(C128, BM_, 1) PP_F2(BM_, 2) PP_F(C128, BM_, 3) PP_F(C128, BM_, 4)
#define PP_8(CFG) template __global__ void pg::gemm_pp_kernel<pg::CFG, pg::A_KMAJOR, pg::B_KMAJOR, pg::E_BF16, 0>(pg::GemmArgs); \
    template __global__ void pg::gemm_pp_kernel<pg::CFG, pg::A_KMAJOR, pg::B_KMAJOR, pg::E_F32, 0>(pg::GemmArgs); \
    template __global__ void pg::gemm_pp_kernel<pg::CFG, pg::A_KMAJOR, pg::B_KMAJOR, pg::E_BF16, 2>(pg::GemmArgs);
PP_8(C8_128) PP_8(C8_96)
#undef PP_8
PP_F5(B_KMAJOR) PP_F5(B_MNMAJOR)
PP_F(C128k, B_KMAJOR, 1) PP_F(C128k, B_KMAJOR, 2) PP_F(C128k, B_KMAJOR, 3) PP_F(C128k, B_KMAJOR, 4)
#undef PP_F5
#undef PP_F2
#undef PP_F
#undef PP_I

// pp_wgrad: out[M][N] (fp32) += alpha * A[K][M]^T . B[K][N] with split-K partial slabs in `ws`
// (>= pdnn_pp_wgrad_ws(M, N, splits) floats) reduced by a second kernel; splits == 1 accumulates in place.
PDNN_API long pdnn_pp_wgrad_ws(int M, int N, int splits) { return splits > 1 ? (long)splits * ((long)M * N + 64) : 0; }
// rowsum (optional, fp32 [M]): += alpha * sum_k A[k][m], fused (the bias gradient of a linear layer beside its
// weight gradient: one extra MFMA per A fragment in the first column tile's items, atomically added per split)
// bn: tile width 128 / 256 (pdnn_pp_wgrad_plan), 0 = pick_bn's choice
PDNN_API int pdnn_pp_wgrad(const bf16_t* A, long lda, const bf16_t* B, long ldb, float* out, long ldc, int M, int N,
                           int K, float alpha, float* ws, int splits, float* rowsum, int bn, hipStream_t st) {
    using namespace pg;
    if (K % PP_SK || M % 8 || N % 8 || splits < 1) return (int)hipErrorInvalidValue;
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K; a.A = A; a.lda = lda; a.B = B; a.ldb = ldb; a.alpha = alpha;
    a.rowsum = rowsum;
    const int nsl = K / PP_SK;
    if (splits > nsl) splits = nsl;
    a.ktiles_per_split = nsl / splits;             // the first nsl % splits splits take one slice more
    a.ksl_rem = nsl % splits;
    if (tune().pp_bn > 0 || (bn != 128 && bn != 256)) bn = pick_bn(a, false, true);
    if (splits == 1) {
        a.C = out; a.ldc = ldc; a.acc_c = 1;
        return launch_bn<A_MNMAJOR, B_MNMAJOR, E_F32>(a, bn, 1, st);
    }
    if (!ws) return (int)hipErrorInvalidValue;
    // slab stride padded by 256 B (pdnn_pp_wgrad_ws): with power-of-two M*N every split of an output falls in
    // the same HBM channel and the reduce crawls
    const long sz = (long)M * N + 64;
    a.C = ws; a.ldc = N; a.sC1 = sz;
    int e = launch_bn<A_MNMAJOR, B_MNMAJOR, E_F32>(a, bn, splits, st);
    if (e) return e;
    // many splits (the long conv-weight-gradient reductions): split-parallel reduce; few (GPT-2): per-output
    if (splits >= 16)
        hipLaunchKernelGGL(pp_slab_reduce_wide_kernel, dim3((unsigned)cdiv((long)M * N / 4, 32)), dim3(256), 0, st,
                           (const float*)ws, sz, splits, out, M, N, ldc, 1);
    else
        hipLaunchKernelGGL(pp_slab_reduce_kernel, dim3(stream_grid((long)M * N / 4, 256)), dim3(256), 0, st,
                           (const float*)ws, sz, splits, out, M, N, ldc, 1);
    PDNN_LAUNCH_RET;
}

// Y[M][N] (bf16) = X[M][K] . W[N][K]^T for a very long reduction: 256 x 256 tiles, K split over `splits`
// work items writing fp32 slabs in `ws` (>= splits * (M * N + 64) floats), summed into bf16 by a second kernel.
PDNN_API int pdnn_pp_gemm_nt_splitk(const bf16_t* X, long ldx, const bf16_t* W, long ldw, bf16_t* Y, long ldy, int M,
                                    int N, int K, float* ws, int splits, hipStream_t st) {
    using namespace pg;
    if (K % PP_SK || N % 8 || ldx % 8 || ldw % 8 || splits < 1 || !ws) return (int)hipErrorInvalidValue;
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K; a.A = X; a.lda = ldx; a.B = W; a.ldb = ldw; a.alpha = 1.f;
    const int nsl = K / PP_SK;
    if (splits > nsl) splits = nsl;
    a.ktiles_per_split = nsl / splits;             // the first nsl % splits splits take one slice more
    a.ksl_rem = nsl % splits;
    const long sz = (long)M * N + 64;             // padded slab stride (see pdnn_pp_wgrad)
    a.C = ws; a.ldc = N; a.sC1 = sz;
    int e = launch_bn<A_KMAJOR, B_KMAJOR, E_F32>(a, 256, splits, st);
    if (e) return e;
    hipLaunchKernelGGL(pp_slab_reduce_bf16_kernel, dim3(stream_grid((long)M * N / 4, 256)), dim3(256), 0, st,
                       (const float*)ws, sz, splits, Y, M, N, ldy);
    PDNN_LAUNCH_RET;
}

// split count for pdnn_pp_gemm_nt_splitk (uneven splits: the first nsl % s take one slice more), minimising
//   rounds x (slices of the longest item + 10) x 0.8 us  +  2 x slab bytes / 5 TB/s
// (256 x 256 tiles, ~0.8 us per 32-deep slice and item round, ~10 slices' worth of per-item prologue / epilogue;
// the slabs are written and read back by the reduction).  The tied LM head's data gradient (8192 x 768 x 50304)
// went from 2 splits (192 of 256 CUs) to 8 (three whole rounds).
PDNN_API int pdnn_pp_splitk_splits(int M, int N, int K) {
    using namespace pg;
    const long tiles = cdiv(M, PP_BM) * cdiv(N, 256);
    const int cus = device_cus(), nsl = K / PP_SK;
    int best = 1;
    double bt = 1e300;
    for (int s = 1; s <= 16; ++s) {
        if (nsl / s < 32) break;
        const double t = (double)cdiv(tiles * s, cus) * (cdiv(nsl, s) + 10) * 0.8
                       + (s > 1 ? 2.0 * s * M * N * 4 / 5e6 : 0.0);
        if (t < bt * 0.999) { bt = t; best = s; }
    }
    return best;
}

// Joint (tile width, K-splits) plan of a linear layer's weight gradient, returned as bn * 1000 + splits: minimises
//   rounds x (slices per item + 10) x u(bn)  +  fp32 traffic of the slabs (split-K) or of the in-place accumulate
// with u = 0.60 / 0.805 us per 32-deep slice per item round for the 128 / 256-wide MN-major tiles and ~5.5 TB/s for
// the slabs, fitted to the GPT-2 shapes (dev/probes/wgrad_sweep.py, gpurun_out/r5_33: e.g. fc 3072 x 768 x 8192
// 256 wide x 6 splits 62.9 us vs 128 x 3 68.6 us).  A forced width (tuning pp_bn) is kept.
// plan_cus > 0: plan for that many CUs (a weight gradient on the side stream beside the data-gradient chain), else
// the device's.
PDNN_API int pdnn_pp_wgrad_plan(int M, int N, int K, int plan_cus) {
    using namespace pg;
    const int cus = plan_cus > 0 && plan_cus < device_cus() ? plan_cus : device_cus();
    const int nsl = K / PP_SK;
    const int force = tune().pp_bn;
    int best_bn = 128, best_s = 1;
    double bt = 1e300;
    for (int bn : {128, 256}) {
        if ((force == 128 || force == 256) && bn != force) continue;
        const long tiles = cdiv(M, PP_BM) * cdiv(N, bn);
        const double u = bn == 128 ? 0.60 : 0.805;
        for (int s = 1; s <= 256; ++s) {
            if (s > 1 && nsl / s < 16) continue;
            const double fp32 = (s > 1 ? (double)s : 1.0) * M * N * 8 / 5.5e6;
            const double t = (double)cdiv(tiles * s, cus) * (cdiv(nsl, s) + 10) * u + fp32;
            if (t < bt * 0.999) { bt = t; best_bn = bn; best_s = s; }
        }
    }
    return best_bn * 1000 + best_s;
}

PDNN_API int pdnn_pp_wgrad_splits(int M, int N, int K) {
    using namespace pg;
    // K-splits (>= 16 slices each, the first nsl % s one slice longer) minimising  rounds x (longest item + ~10 slices of
    // per-item prologue/epilogue), with a 4% per-split surcharge for the fp32 slab traffic and reduction:
    // a split count that spills a few items into a second round of the persistent grid costs as much as
    // halving it (GPT-2 fc / fc2: 4 -> 2 splits, tools/pp_check.py wg_* rows)
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K;
    const int bn = pick_bn(a, false, true);
    const long tiles = cdiv(M, PP_BM) * cdiv(N, bn);
    const int cus = device_cus();
    const int nsl = K / PP_SK;
    int best = 1;
    double bt = 1e300;
    for (int s = 1; s <= 32; ++s) {
        if (s > 1 && nsl / s < 16) continue;
        const double t = (double)cdiv(tiles * s, cus) * (cdiv(nsl, s) + 10) * (1.0 + 0.04 * (s - 1));
        if (t < bt) { bt = t; best = s; }
    }
    return best;
}

// K-splits for the long-reduction weight gradients of 1x1 convs (K = pixels, 10^4..10^5 slices, few output
// tiles): minimise  max(latency term, operand-traffic term) + slab term  [us], fitted to the ResNet-50 stage-2..4
// shapes (tools/bench_wgrad1x1.py, gpurun_out/r3_38): ~0.65 us per slice per item round plus ~10 slices of
// per-item overhead, operand bytes at ~6 TB/s, fp32 slab written and re-read at ~4 TB/s; up to 256 splits.
PDNN_API int pdnn_pp_wgrad_splits_long(int M, int N, int K) {
    using namespace pg;
    GemmArgs a{};
    a.M = M; a.N = N; a.K = K;
    const int bn = pick_bn(a, false, true);
    const long tiles = cdiv(M, PP_BM) * cdiv(N, bn);
    const int cus = device_cus();
    const int nsl = K / PP_SK;
    // operand bytes: a tile wider than the matrix re-reads clamped rows from L2, so count the real extent
    const double mem = (double)tiles * nsl * ((M < PP_BM ? M : PP_BM) + (N < bn ? N : bn)) * 64 / 6e6;
    int best = 1;
    double bt = 1e300;
    for (int s = 1; s <= 256; ++s) {
        if (nsl % s || (s > 1 && nsl / s < 16)) continue;
        const double lat = (double)cdiv(tiles * s, cus) * (nsl / s + 10) * 0.65;
        const double t = (lat > mem ? lat : mem) + (s > 1 ? 2.0 * s * M * N * 4 / 4e6 : 0.0);
        if (t < bt) { bt = t; best = s; }
    }
    return best;
}

// phase trace buffer for the next pp launches (null = off): 2 * grid * 64 int64 timestamps (100 MHz)
PDNN_API void pdnn_set_pp_trace(long long* buf) { pg::g_pp_trace = buf; }

// force a tile width (0 = automatic); returns the previous setting.  A/B experiments and tests.
PDNN_API int pdnn_set_pp_bn(int bn) {
    const int old = pg::tune().pp_bn;
    pg::tune().pp_bn = bn;
    return old;
}
