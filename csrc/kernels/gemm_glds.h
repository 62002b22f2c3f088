// Included by gemm_mfma.hip inside its anonymous namespace (uses GemmArgs, FastDiv, fragment readers).
//
// glds engine: the large-tile GEMM / implicit-GEMM-conv kernel for gfx950.
//
//  * Block tile BM x BN x 64 with BM = 256 and BN in {256, 128, 64}; WM x WN waves (8, 8, 4 waves),
//    wave tile (BM/WM) x (BN/WN) of 16x16x32 bf16 MFMA fragments (MI355X_MICROARCH.md: 16x16x32 holds a
//    higher clock than 32x32x16 on random data).
//  * Both operands are staged global -> LDS with `global_load_lds_dwordx4` (glds): no VGPR round trip and
//    no ds_write pass, 2 LDS buffers, one barrier per K-step, the next tile's glds in flight during this
//    tile's MFMAs (cdna_hip_programming.md §5 "glds vs register staging").  One glds wave-instruction
//    fills 1 KiB of LDS = 8 K-major rows or 512/BN... MN-major k-rows; the image is lane-linear and the bank
//    swizzle is applied on the per-lane GLOBAL source address (guide rule 21).
//  * Gathers are free with glds: the global address is per lane.  Implicit-GEMM conv operands compute
//    the address of each lane's 16-byte piece (8 channels of one pixel and tap) per K-step; padded taps
//    read a 16-byte zero page instead of being predicated.  Supported: the forward im2col gather
//    (A_CONV, C % 64 == 0), the transposed gather of the data gradient per parity class (A_CONVT,
//    Ko % 64 == 0), weights as [(r,s,ko)][c] (B_WT) and the weight-gradient im2col (B_IM2COL).
//  * Epilogues: alpha / bias / ReLU / GELU(+pre-activation) / dGELU / residual, BatchNorm forward partial
//    statistics, BatchNorm-backward masking + statistics, parity-class row scatter, fp32 output, and
//    split-K fp32 atomics through an LDS C-stage (optionally transposed, for the swapped weight gradient).
//  * The fused BN-affine+ReLU operand prologue is NOT possible here (glds data never passes through
//    registers); those convolutions keep the register-staged 128-tile kernel.

__device__ __attribute__((aligned(16))) uint4 g_zero16[4];      // zero page for padded gathers

constexpr int GBM = 256;
constexpr int GCST_ROWS = 64;                                   // atomic epilogue: C stage rows per round

template <int BN>
constexpr int glds_smem() {
    const int ops = 2 * (GBM + BN) * BK * 2;
    const int cst = GCST_ROWS * (BN + CPAD) * 4;
    return ops > cst ? ops : cst;
}

__device__ __forceinline__ void glds16(const void* src, bf16_t* dst) {
    __builtin_amdgcn_global_load_lds(src, (lds_void*)dst, 16, 0, 0);
}

// ---------------------------------------------------------------------------------------------------
// K-major operand (rows = m or n, 64 k per row).  One instruction = 8 rows.  KIND 0 plain, 1 conv
// gather, 2 conv-transposed gather (parity class).
// ---------------------------------------------------------------------------------------------------
template <int ROWS, int NWAVES, int KIND>
struct GK {
    static constexpr int NI = ROWS / 8 / NWAVES;
    const bf16_t* base[NI];
    int hb[NI], wb[NI];
    int coff;                 // this lane's chunk column offset (elements), same for all its rows
    int kcur;                 // plain: current k
    int r, s, c0;             // conv: current tap (r, s) / class tap (ir, is) and channel block

    __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p, long ld, int rows_total, int row0,
                                         int wave, int lane, int kt0) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int rr = 8 * (wave * NI + i) + (lane >> 3);
            const int row = row0 + rr;
            const bool v = row < rows_total;
            const int rw = v ? row : rows_total - 1;
            if constexpr (KIND == 0) {
                base[i] = p + (long)rw * ld;
            } else {
                const ConvGeom& g = a.g;
                const uint32_t n = fdiv((uint32_t)rw, g.dHW);
                const uint32_t rem = (uint32_t)rw - n * g.dHW.d;
                const uint32_t y = fdiv(rem, g.dW);
                const uint32_t x = rem - y * g.dW.d;
                if constexpr (KIND == 1) {
                    hb[i] = v ? (int)y * g.st - g.pad : -(1 << 28);
                    wb[i] = (int)x * g.st - g.pad;
                    base[i] = p + (long)n * g.H * g.W * g.C;
                } else {
                    hb[i] = v ? (int)y * g.st + g.ph + g.pad : -(1 << 28);
                    wb[i] = (int)x * g.st + g.pw + g.pad;
                    base[i] = p + (long)n * g.Ho * g.Wo * g.Ko;
                }
            }
            // chunk position (lane & 7) holds global chunk (lane & 7) ^ ((rr >> 1) & 7); rr & 15 is the
            // same for every instruction of this lane only modulo 8 rows -> compute per row below
        }
        coff = 0;
        kcur = kt0 * BK;
        if constexpr (KIND == 1) {
            const int rs = kcur / a.g.C;
            c0 = kcur - rs * a.g.C;
            r = rs / a.g.S;
            s = rs - r * a.g.S;
        } else if constexpr (KIND == 2) {
            const int rs = kcur / a.g.Ko;
            c0 = kcur - rs * a.g.Ko;
            r = rs / a.g.Sc;
            s = rs - r * a.g.Sc;
        }
    }

    __device__ __forceinline__ void issue(const GemmArgs& a, bf16_t* img, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int rr = 8 * (wave * NI + i) + (lane >> 3);
            const int ch = ((lane & 7) ^ ((rr >> 1) & 7)) * 8;
            const void* src;
            if constexpr (KIND == 0) {
                src = base[i] + kcur + ch;
            } else if constexpr (KIND == 1) {
                const ConvGeom& g = a.g;
                const int h = hb[i] + r, w = wb[i] + s;
                const bool ok = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
                src = ok ? (const void*)(base[i] + ((long)h * g.W + w) * g.C + c0 + ch) : (const void*)g_zero16;
            } else {
                const ConvGeom& g = a.g;
                int th = hb[i] - (g.r0 + g.st * r), tw = wb[i] - (g.s0 + g.st * s);
                bool ok = th >= 0 && tw >= 0;
                if (g.st != 1) { th /= g.st; tw /= g.st; }     // exact by construction of the parity class
                ok = ok && th < g.Ho && tw < g.Wo;
                src = ok ? (const void*)(base[i] + ((long)th * g.Wo + tw) * g.Ko + c0 + ch) : (const void*)g_zero16;
            }
            glds16(src, img + (wave * NI + i) * 512);
        }
        kcur += BK;
        if constexpr (KIND == 1) {
            c0 += BK;
            if (c0 >= a.g.C) { c0 = 0; if (++s == a.g.S) { s = 0; ++r; } }
        } else if constexpr (KIND == 2) {
            c0 += BK;
            if (c0 >= a.g.Ko) { c0 = 0; if (++s == a.g.Sc) { s = 0; ++r; } }
        }
    }
};

// ---------------------------------------------------------------------------------------------------
// MN-major operand ([64 k-rows][W] image).  One instruction = 512 / W k-rows.  KIND 0 plain [k][ld],
// 1 weights as [(ir, is, ko)][c] of a parity class (B_WT), 2 im2col of NHWC input, k = output pixel.
// ---------------------------------------------------------------------------------------------------
template <int W, int NWAVES, int KIND>
struct GM {
    static constexpr int CPR = W / 8;               // chunks per image row
    static constexpr int RPI = 64 / CPR;            // image rows per instruction (8 lanes x ... ) = 512 / W
    static constexpr int NI = 64 / RPI / NWAVES;    // instructions per wave per K-step
    const bf16_t* p;
    long ld;
    int col;                                        // this lane's global column (chunk start)
    int kbase;
    int cr, cs, cc;                                 // im2col: the column's (r, s, c)

    __device__ __forceinline__ static int swz(int krow) {
        if constexpr (W >= 128) return ((krow & 3) | ((krow >> 1) & 4)) << 1;
        else return (((krow >> 1) & 1) | ((krow >> 2) & 2)) << 1;
    }
    __device__ __forceinline__ int krow_of(int wave, int i, int lane) const {
        return (wave * NI + i) * RPI + lane / CPR;
    }

    __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* p_, long ld_, int cols_total, int col0,
                                         int wave, int lane, int kt0) {
        p = p_;
        ld = ld_;
        kbase = kt0 * BK;
        // every instruction of this lane covers the same column chunk position; the swizzle depends on
        // the k-row, which differs per instruction -> columns are computed per instruction in issue()
        col = col0;
        (void)cols_total;
        if constexpr (KIND == 2) { cr = cs = cc = 0; }
    }

    __device__ __forceinline__ void issue(const GemmArgs& a, bf16_t* img, int wave, int lane, int cols_total) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int kr = krow_of(wave, i, lane);
            const int c = (lane % CPR) ^ swz(kr);
            const int cl = min(col + 8 * c, cols_total - 8);
            const int k = kbase + kr;
            const void* src;
            if constexpr (KIND == 0) {
                src = p + (long)k * ld + cl;
            } else if constexpr (KIND == 1) {
                const ConvGeom& g = a.g;
                const uint32_t rs = fdiv((uint32_t)k, g.dKo);
                const int ko = k - (int)(rs * g.Ko);
                const uint32_t ir = fdiv(rs, g.dSc);
                const int rr = g.r0 + g.st * (int)ir, ss = g.s0 + g.st * (int)(rs - ir * g.Sc);
                src = p + ((long)ko * g.R * g.S + rr * g.S + ss) * g.C + cl;
            } else {
                const ConvGeom& g = a.g;
                const uint32_t rs = fdiv((uint32_t)cl, g.dC);
                const int c_ = cl - (int)(rs * g.C);
                const uint32_t r_ = fdiv(rs, g.dS);
                const int s_ = (int)(rs - r_ * g.S);
                const bool kv = k < a.K;
                const uint32_t kk = kv ? (uint32_t)k : 0u;
                const uint32_t n = fdiv(kk, g.dHW);
                const uint32_t rem = kk - n * g.dHW.d;
                const uint32_t yo = fdiv(rem, g.dW);
                const uint32_t xo = rem - yo * g.dW.d;
                const int hi = (int)yo * g.st - g.pad + (int)r_, wi = (int)xo * g.st - g.pad + s_;
                const bool ok = kv && (unsigned)hi < (unsigned)g.H && (unsigned)wi < (unsigned)g.W;
                src = ok ? (const void*)(p + (((long)n * g.H + hi) * g.W + wi) * g.C + c_) : (const void*)g_zero16;
            }
            glds16(src, img + (wave * NI + i) * 512);
        }
        kbase += BK;
    }
};

template <int AM, int ROWS, int NW> struct GASel;
template <int ROWS, int NW> struct GASel<A_KMAJOR, ROWS, NW> { using T = GK<ROWS, NW, 0>; static constexpr bool K = true; };
template <int ROWS, int NW> struct GASel<A_CONV, ROWS, NW> { using T = GK<ROWS, NW, 1>; static constexpr bool K = true; };
template <int ROWS, int NW> struct GASel<A_CONVT, ROWS, NW> { using T = GK<ROWS, NW, 2>; static constexpr bool K = true; };
template <int ROWS, int NW> struct GASel<A_MNMAJOR, ROWS, NW> { using T = GM<ROWS, NW, 0>; static constexpr bool K = false; };
template <int ROWS, int NW> struct GASel<A_IM2COL, ROWS, NW> { using T = GM<ROWS, NW, 2>; static constexpr bool K = false; };
template <int BMODE, int W, int NW> struct GBSel;
template <int W, int NW> struct GBSel<B_KMAJOR, W, NW> { using T = GK<W, NW, 0>; static constexpr bool K = true; };
template <int W, int NW> struct GBSel<B_MNMAJOR, W, NW> { using T = GM<W, NW, 0>; static constexpr bool K = false; };
template <int W, int NW> struct GBSel<B_WT, W, NW> { using T = GM<W, NW, 1>; static constexpr bool K = false; };
template <int W, int NW> struct GBSel<B_IM2COL, W, NW> { using T = GM<W, NW, 2>; static constexpr bool K = false; };

template <bool KM, typename L>
__device__ __forceinline__ void gissue(L& l, const GemmArgs& a, bf16_t* img, int wave, int lane, int extent) {
    if constexpr (KM) l.issue(a, img, wave, lane);
    else l.issue(a, img, wave, lane, extent);
}

template <int BN> struct GWaves;                      // wave arrangement per tile width
template <> struct GWaves<256> { static constexpr int WM = 2, WN = 4; };
template <> struct GWaves<128> { static constexpr int WM = 4, WN = 2; };
template <> struct GWaves<64> { static constexpr int WM = 4, WN = 1; };

// fp8 fragment of the block-scaled 16x16x128 MFMA: lane l holds 32 consecutive k bytes
// [32 (l >> 4), +32) of row (row0 + (l & 15)) = 16-byte chunks 2g, 2g+1 of the 128-byte image row
typedef __attribute__((ext_vector_type(8))) int v8i_t;
__device__ __forceinline__ v8i_t frag_fp8(const bf16_t* img, int row, int lane) {
    const int g = lane >> 4;
    const u16x8_t lo = *reinterpret_cast<const u16x8_t*>(img + kimg_off(row, 2 * g));
    const u16x8_t hi = *reinterpret_cast<const u16x8_t*>(img + kimg_off(row, 2 * g + 1));
    typedef __attribute__((ext_vector_type(4))) int v4i_t;
    const v4i_t a = __builtin_bit_cast(v4i_t, lo), b = __builtin_bit_cast(v4i_t, hi);
    return v8i_t{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

// DT = 1: fp8 (OCP e4m3) operands, both K-major; the caller passes every K / ld in units of 2 fp8
// (the loaders move bytes), so one 64-"element" K-step is 128 fp8 = one block-scaled MFMA step
// (unit block scales: per-tensor scales are applied in the epilogue through alpha_ptr).
template <int AM, int BMODE, int EM, int BN, int DT = 0>
__global__ void __launch_bounds__(GWaves<BN>::WM * GWaves<BN>::WN * 64)
gemm_glds_kernel(GemmArgs a) {
    constexpr int WM = GWaves<BN>::WM, WN = GWaves<BN>::WN, NWAVE = WM * WN, NTH = NWAVE * 64;
    constexpr int WTM = GBM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
    constexpr int IMA = GBM * BK, IMB = BN * BK;      // bf16 elements per operand image
    using LA = typename GASel<AM, GBM, NWAVE>::T;
    using LB = typename GBSel<BMODE, BN, NWAVE>::T;
    constexpr bool AK = GASel<AM, GBM, NWAVE>::K, BKm = GBSel<BMODE, BN, NWAVE>::K;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const sbase = reinterpret_cast<bf16_t*>(smem);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    if (gridDim.y > 1) {
        const int z = blockIdx.y, z1 = z / a.nb2, z2 = z - z1 * a.nb2;
        a.A += z1 * a.sA1 + z2 * a.sA2;
        a.B += z1 * a.sB1 + z2 * a.sB2;
        a.C = (void*)((char*)a.C + (z1 * a.sC1 + z2 * a.sC2) * (EM == E_BF16 ? 2 : 4));
        if (a.ep_res) a.ep_res += z1 * a.sC1 + z2 * a.sC2;
    }
    const int tiles_m = (a.M + GBM - 1) / GBM, tiles_n = (a.N + BN - 1) / BN;
    const int ntiles = tiles_m * tiles_n;
    const int ktiles = (a.K + BK - 1) / BK;
    // Grid-stride over output tiles (block b takes tiles b, b + G, ...; the launcher uses one block per tile: a
    // persistent grid measured slower than the hardware dispatcher on every shape tried); the next tile's first
    // K-step is issued into the free LDS buffer before this tile's epilogue.
    int cur = 0;
    bool pre = false;
    LA la;
    LB lb;
    for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int t = xcd_remap(tile, ntiles);
    const int tm = t / tiles_n, tn = t % tiles_n;
    const int m0 = tm * GBM, n0 = tn * BN;

    int kt0 = blockIdx.z * a.ktiles_per_split;
    int kt1 = min(ktiles, kt0 + a.ktiles_per_split);
    if (a.causal == 1 && n0 >= m0 + GBM) continue;
    if (a.causal == 2) kt1 = min(kt1, (m0 + GBM + BK - 1) / BK);
    if (a.causal == 3) kt0 = max(kt0, m0 / BK);
    if (kt0 >= kt1) continue;

    if (!pre) {
        la.init(a, a.A, a.lda, a.M, m0, wave, lane, kt0);
        lb.init(a, a.B, a.ldb, a.N, n0, wave, lane, kt0);
        gissue<AK>(la, a, sbase + cur * (IMA + IMB), wave, lane, a.M);
        gissue<BKm>(lb, a, sbase + cur * (IMA + IMB) + IMA, wave, lane, a.N);
    }
    pre = false;

    f32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    for (int kt = kt0; kt < kt1; ++kt) {
        if (kt + 1 < kt1) {
            bf16_t* nb = sbase + (cur ^ 1) * (IMA + IMB);
            gissue<AK>(la, a, nb, wave, lane, a.M);
            gissue<BKm>(lb, a, nb + IMA, wave, lane, a.N);
        }
        const bf16_t* A_ = sbase + cur * (IMA + IMB);
        const bf16_t* B_ = A_ + IMA;
        if constexpr (DT == 1) {
            v8i_t bq[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) bq[f] = frag_fp8(B_, wn * WTN + f * 16 + (lane & 15), lane);
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
                const v8i_t aq = frag_fp8(A_, wm * WTM + fm * 16 + (lane & 15), lane);
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                        bq[fn], aq, acc[fm][fn], 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
            }
        }
#pragma unroll
        for (int ks = 0; ks < (DT == 1 ? 0 : 2); ++ks) {
            bf16x8_t bfr[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) {
                if constexpr (BKm) bfr[f] = frag_kmajor(B_, wn * WTN + f * 16 + (lane & 15), ks, lane);
                else bfr[f] = frag_mnmajor<BN>(B_, wn * WTN + f * 16, ks, lane);
            }
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
                bf16x8_t af;
                if constexpr (AK) af = frag_kmajor(A_, wm * WTM + fm * 16 + (lane & 15), ks, lane);
                else af = frag_mnmajor<GBM>(A_, wm * WTM + fm * 16, ks, lane);
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af, acc[fm][fn], 0, 0, 0);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        cur ^= 1;
    }
    if constexpr (EM != E_ATOMIC) {     // (the atomic epilogue stages C through the LDS buffers)
        const int nt = tile + gridDim.x;
        if (nt < ntiles && a.causal == 0) {
            const int t2 = xcd_remap(nt, ntiles);
            const int kt0n = blockIdx.z * a.ktiles_per_split;
            la.init(a, a.A, a.lda, a.M, (t2 / tiles_n) * GBM, wave, lane, kt0n);
            lb.init(a, a.B, a.ldb, a.N, (t2 % tiles_n) * BN, wave, lane, kt0n);
            gissue<AK>(la, a, sbase + cur * (IMA + IMB), wave, lane, a.M);
            gissue<BKm>(lb, a, sbase + cur * (IMA + IMB) + IMA, wave, lane, a.N);
            pre = true;
        }
    }

    // ---------------- epilogue: lane holds C[m0 + wm*WTM + fm*16 + lm][n0 + wn*WTN + fn*16 + 4*lg + j]
    const int lm = lane & 15, lg = lane >> 4;
    if (a.alpha_ptr) a.alpha *= *a.alpha_ptr;      // device-side scale (fp8 dequantisation)
    if constexpr (EM == E_ATOMIC) {
        // rounds of GCST_ROWS rows through an fp32 LDS stage -> 256-byte contiguous atomic wave-instructions
        float* cs = reinterpret_cast<float*>(smem);
        constexpr int LDC_S = BN + CPAD;
        float* C = reinterpret_cast<float*>(a.C);
#pragma unroll 1
        for (int r0 = 0; r0 < GBM; r0 += GCST_ROWS) {
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
                const int rl = wm * WTM + fm * 16 - r0;       // wave-uniform
                if (rl >= 0 && rl < GCST_ROWS) {
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
                        *reinterpret_cast<f32x4_t*>(cs + (rl + lm) * LDC_S + wn * WTN + fn * 16 + 4 * lg) = acc[fm][fn];
                }
            }
            __syncthreads();
            if (a.transC) {
                // C^T[n][m]: each wave sweeps columns, its lanes the stage's rows (64 contiguous floats)
                for (int c = wave; c < BN; c += NWAVE) {
                    const int n = n0 + c;
                    if (n >= a.N) break;
                    const int m = m0 + r0 + lane;
                    if (m < a.M) atomicAdd(C + (long)n * a.ldc + m, a.alpha * cs[lane * LDC_S + c]);
                }
            } else {
                for (int r = wave; r < GCST_ROWS; r += NWAVE) {
                    const int m = m0 + r0 + r;
                    if (m >= a.M) break;
#pragma unroll
                    for (int q = 0; q < BN / 64; ++q) {
                        const int c = q * 64 + lane;
                        const int n = n0 + c;
                        if (n < a.N) atomicAdd(C + (long)m * a.ldc + n, a.alpha * cs[r * LDC_S + c]);
                    }
                }
            }
            __syncthreads();
        }
        continue;
    } else {
        const bool bnb = a.ep_x != nullptr;
        const bool want_stats = EM == E_BF16 && a.stats != nullptr;
        // per-column partial statistics, accumulated over the wave's rows, one slab row pair per 64 rows
        float s_[FN][4], q_[FN][4];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn)
#pragma unroll
            for (int j = 0; j < 4; ++j) s_[fn][j] = q_[fn][j] = 0.f;
        static_for<0, FM>([&](auto FMC) {
            constexpr int fm = decltype(FMC)::value;
            const int m = m0 + wm * WTM + fm * 16 + lm;
            const bool mv = m < a.M;
            long orow = m;
            if (a.scatter && mv) {
                const uint32_t nn = fdiv((uint32_t)m, a.g.dHW);
                const uint32_t rem = (uint32_t)m - nn * a.g.dHW.d;
                const uint32_t hc = fdiv(rem, a.g.dW);
                const uint32_t wc = rem - hc * a.g.dW.d;
                orow = ((long)nn * a.g.H + hc * a.g.st + a.g.ph) * a.g.W + wc * a.g.st + a.g.pw;
            }
            uint32_t pk[FN][2];
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int n = n0 + wn * WTN + fn * 16 + 4 * lg;
                const bool n4 = n + 4 <= a.N, ok = mv && n4;
                const long off = orow * a.ldc + n;
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    v[j] = acc[fm][fn][j] * a.alpha;
                    if (a.bias) v[j] += n4 ? a.bias[n + j] : 0.f;
                    if (a.relu == 1) v[j] = fmaxf(v[j], 0.f);
                }
                if constexpr (EM == E_BF16) {
                    if (a.relu == 2) {
                        u16x4_t pre;
#pragma unroll
                        for (int j = 0; j < 4; ++j) pre[j] = f2bf(v[j]);
                        if (a.ep_aux && ok) *reinterpret_cast<u16x4_t*>(a.ep_aux + off) = pre;
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = gelu_tanh(bf2f(pre[j]));
                    }
                    if (a.ep_dgelu && ok) {
                        const u16x4_t u = *reinterpret_cast<const u16x4_t*>(a.ep_dgelu + off);
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] *= gelu_tanh_grad(bf2f(u[j]));
                    }
                    if (a.ep_res && ok) {
                        const u16x4_t r = *reinterpret_cast<const u16x4_t*>(a.ep_res + off);
                        const uint32_t mb = a.ep_rmask ? (uint32_t)(a.ep_rmask[off >> 3] >> (off & 4)) : 0xFu;
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] += ((mb >> j) & 1) ? bf2f(r[j]) : 0.f;
                    }
                    if (bnb) {
                        // BN coefficients re-read per fragment (L1-resident): keeping them live across the
                        // fragment loop pushes the 256-wide variant into scratch
                        u16x4_t tv = {0, 0, 0, 0};
                        float4 mu = {0, 0, 0, 0}, is = mu, ms = mu, mh = mu;
                        if (ok) {
                            tv = *reinterpret_cast<const u16x4_t*>(a.ep_x + off);
                            mu = *reinterpret_cast<const float4*>(a.ep_mean + n);
                            is = *reinterpret_cast<const float4*>(a.ep_invstd + n);
                            ms = *reinterpret_cast<const float4*>(a.ep_mscale + n);
                            mh = *reinterpret_cast<const float4*>(a.ep_mshift + n);
                        }
                        const float mua[4] = {mu.x, mu.y, mu.z, mu.w}, isa[4] = {is.x, is.y, is.z, is.w};
                        const float msa[4] = {ms.x, ms.y, ms.z, ms.w}, mha[4] = {mh.x, mh.y, mh.z, mh.w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float tt = bf2f(tv[j]);
                            const float gm = (ok && fmaf(tt, msa[j], mha[j]) > 0.f) ? bf2f(f2bf(v[j])) : 0.f;
                            v[j] = gm;
                            s_[fn][j] += gm;
                            q_[fn][j] += ok ? gm * (tt - mua[j]) * isa[j] : 0.f;
                        }
                    } else if (want_stats && ok) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float rr = bf2f(f2bf(v[j]));
                            s_[fn][j] += rr;
                            q_[fn][j] += rr * rr;
                        }
                    }
                    pk[fn][0] = pk2bf(v[0], v[1]);
                    pk[fn][1] = pk2bf(v[2], v[3]);
                } else {
                    if (!mv || n >= a.N) continue;
                    float* C = reinterpret_cast<float*>(a.C) + off;
                    if (n4 && (a.ldc & 3) == 0) *reinterpret_cast<float4*>(C) = make_float4(v[0], v[1], v[2], v[3]);
                    else for (int j = 0; j < 4 && n + j < a.N; ++j) C[j] = v[j];
                }
            }
            if constexpr (EM == E_BF16) {
                // 16-byte stores: permlane16 swap pairs fragments (fn, fn+1) (T21)
#pragma unroll
                for (int fp = 0; fp < FN / 2; ++fp) {
                    const auto s0 = __builtin_amdgcn_permlane16_swap(pk[2 * fp][0], pk[2 * fp + 1][0], false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(pk[2 * fp][1], pk[2 * fp + 1][1], false, false);
                    const int n = n0 + wn * WTN + (2 * fp + (lg & 1)) * 16 + 8 * (lg >> 1);
                    if (mv && n + 8 <= a.N) {
                        *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(a.C) + orow * a.ldc + n) =
                            make_uint4(s0[0], s1[0], s0[1], s1[1]);
                    } else if (mv && n < a.N) {
                        const uint32_t w4[4] = {s0[0], s1[0], s0[1], s1[1]};
                        bf16_t* C = reinterpret_cast<bf16_t*>(a.C) + orow * a.ldc + n;
                        for (int j = 0; j < 8 && n + j < a.N; ++j) C[j] = (bf16_t)(w4[j >> 1] >> (16 * (j & 1)));
                    }
                }
                if constexpr (FN % 2) {        // FN == 1 (BN = 64 with 1 wave column): plain 8-byte stores
                    const int n = n0 + wn * WTN + 4 * lg;
                    bf16_t* C = reinterpret_cast<bf16_t*>(a.C) + orow * a.ldc + n;
                    if (mv && n + 4 <= a.N) *reinterpret_cast<uint2*>(C) = make_uint2(pk[FN - 1][0], pk[FN - 1][1]);
                }
                // statistics: flush one slab row pair per 64 rows (4 fragments) of the wave
                if ((want_stats || bnb) && (fm % 4 == 3 || fm == FM - 1)) {
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            s_[fn][j] = row16_sum(s_[fn][j]);
                            q_[fn][j] = row16_sum(q_[fn][j]);
                        }
                    const int grp = m0 + wm * WTM + (fm / 4) * 64;           // first row of these 64
                    const int slab_row = a.stats_row0 + grp / 64;
                    // the slab has one row pair per 64 rows of M rounded up to 128 (the 128-tile layout)
                    if (grp < ((a.M + 127) / 128) * 128) {
#pragma unroll
                        for (int fn = 0; fn < FN; ++fn) {
                            const int n = n0 + wn * WTN + fn * 16 + 4 * lg;
                            float* ps = stat_row(a.stats, slab_row, a.N) + n;
                            stat_add_frag(ps, ps + a.N, lane, s_[fn], q_[fn], n + (lm & 3) < a.N);
                        }
                    }
#pragma unroll
                    for (int fn = 0; fn < FN; ++fn)
#pragma unroll
                        for (int j = 0; j < 4; ++j) s_[fn][j] = q_[fn][j] = 0.f;
                }
            }
        });
    }
    }   // tile loop
}

template <int AM, int BMODE, int EM, int BN, int DT = 0>
int launch_glds_w(const GemmArgs& a, int splits, hipStream_t st, int batch) {
    constexpr int NTH = GWaves<BN>::WM * GWaves<BN>::WN * 64;
    constexpr int SM = glds_smem<BN>();
    static bool attr = false;
    if (!attr) {
        attr = true;
        (void)hipFuncSetAttribute((const void*)gemm_glds_kernel<AM, BMODE, EM, BN, DT>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, SM);
    }
    const int tiles = (int)(cdiv(a.M, GBM) * cdiv(a.N, BN));
    hipLaunchKernelGGL((gemm_glds_kernel<AM, BMODE, EM, BN, DT>), dim3(tiles, batch, splits), dim3(NTH), SM, st, a);
    PDNN_LAUNCH_RET;
}

// tile width for N: the widest of {256, 128, 64} that does not leave a mostly-empty last column tile
inline int glds_bn(int N) {
    if (N % 256 == 0 || N >= 1024) return 256;     // at most 1/8 of the last column tile wasted
    if (N % 128 == 0 || N > 512) return 128;
    return 64;
}

template <int AM, int BMODE, int EM>
int launch_glds(const GemmArgs& a, int splits, hipStream_t st, int batch, int bn) {
    if (bn == 256) return launch_glds_w<AM, BMODE, EM, 256>(a, splits, st, batch);
    if (bn == 128) return launch_glds_w<AM, BMODE, EM, 128>(a, splits, st, batch);
    return launch_glds_w<AM, BMODE, EM, 64>(a, splits, st, batch);
}

// Operand-shape conditions of the glds engine (the epilogue features are all supported).
template <int AM, int BMODE>
bool glds_operands_ok(const GemmArgs& a) {
    if (a.M < 8 || a.N < 8 || a.N % 8) return false;
    if constexpr (AM == A_KMAJOR || AM == A_MNMAJOR) { if (a.lda % 8) return false; }
    if constexpr (AM == A_MNMAJOR || AM == A_IM2COL) { if (a.M % 8) return false; }
    if constexpr (BMODE == B_KMAJOR || BMODE == B_MNMAJOR) { if (a.ldb % 8) return false; }
    // K-major operands load whole 64-wide k slices: K must be a multiple of 64 (no partial k tile)
    if constexpr (AM == A_KMAJOR || BMODE == B_KMAJOR) { if (a.K % BK) return false; }
    if constexpr (AM == A_CONV) { if (a.g.C % BK) return false; }
    if constexpr (AM == A_CONVT || BMODE == B_WT) { if (a.g.Ko % BK) return false; }
    if constexpr (AM == A_MNMAJOR || BMODE == B_MNMAJOR || BMODE == B_WT) { if (a.K % BK) return false; }
    if constexpr (BMODE == B_IM2COL || AM == A_IM2COL) { if (a.g.C % 8) return false; }
    return true;
}
