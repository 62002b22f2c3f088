// Shared definitions of the GEMM engines (gemm_mfma.hip: register-staged + glds engines and the C API;
// gemm_pp.hip: the ping-pong engine).  Named namespace so GemmArgs can cross translation units.
#pragma once
#include "common.h"

namespace pg {

constexpr int BK = 64;
constexpr int NT = 256;

enum AMode { A_KMAJOR = 0, A_MNMAJOR = 1, A_CONV = 2, A_CONVT = 3, A_IM2COL = 4 };
enum BMode { B_KMAJOR = 0, B_MNMAJOR = 1, B_WT = 2, B_IM2COL = 3 };
enum EMode { E_BF16 = 0, E_F32 = 1, E_ATOMIC = 2 };

// Granlund-Montgomery unsigned division by a runtime-invariant divisor (valid for n < 2^31).
struct FastDiv {
    uint32_t d, m, s;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return (__umulhi(n, f.m) + n) >> f.s;
}

struct ConvGeom {
    int Nimg, H, W, C;      // activation tensor of the gather (NHWC)
    int Ho, Wo, R, S;       // the "other" spatial extent and filter size
    int st, pad;
    int Ko;                 // output channels (for A_CONVT / B_WT reduction index)
    // transposed-conv parity class (dgrad with stride > 1 is split into st*st dense sub-problems):
    // output pixels h = hc*st + ph, taps r = r0 + st*ir (ir < Rc); identical to a plain conv when st == 1
    int ph, pw, r0, s0, Sc;
    FastDiv dHW, dW, dC, dS, dKo, dSc;  // divisors used by the gathers
};

struct GemmArgs {
    int M, N, K;
    const bf16_t* A; long lda;
    const bf16_t* B; long ldb;
    ConvGeom g;
    const float* pro_scale;   // optional fused prologue  x -> relu(x*scale[c] + shift[c])
    const float* pro_shift;
    void* C; long ldc;
    float alpha;
    const float* bias;        // per-column bias (E_BF16 / E_F32)
    int relu;                 // epilogue activation: 0 none, 1 ReLU, 2 GELU (tanh form)
    float* stats;             // [gridM*2 rows][2][N] per-wave-row partial (sum, sumsq), or null
    int ktiles_per_split;     // split-K (grid.z)
    int ksl_rem;              // pp engine: the first ksl_rem K-splits take one slice more (uneven splits)
    float* rowsum;            // pp engine E_F32: += alpha * sum_k A[m][k] per output row m (fused bias gradient)
    int scatter;              // epilogue rows are parity-class pixels of dIn (A_CONVT with stride > 1)
    int stats_row0;           // first slab row of this launch (parity-class launches share one slab)
    int transC;               // E_ATOMIC: accumulate C^T (C[n * ldc + m])
    // batched GEMM (grid.y = nb1 * nb2): operand offsets z1 * s*1 + z2 * s*2 (elements), z = z1 * nb2 + z2
    int nb2;
    long sA1, sA2, sB1, sB2, sC1, sC2;
    // causal attention structure (square T x T operands, row = query, col = key):
    //  1: C tiles strictly above the diagonal are skipped (S = Q K^T; never read by the softmax)
    //  2: reduction limited to k < m0 + BM   (A = P or dS [q][k], lower triangular: P V, dS K)
    //  3: reduction starts at k >= m0        (A = P^T / dS^T, upper triangular: P^T dO, dS^T Q)
    int causal;
    int stage_store;          // 128-row kernel: bf16 epilogue stores staged through LDS (full-row writes)
    // epilogue fusions (E_BF16): residual add, and BN-backward masking + statistics (see epilogue)
    const bf16_t* ep_res;
    const uint8_t* ep_rmask;  // optional: residual masked by bit (n & 7) of ep_rmask[(row*ldc + n) >> 3] (ReLU bits)
    const bf16_t* ep_x;
    const float *ep_mean, *ep_invstd, *ep_mscale, *ep_mshift;
    const float* alpha_ptr;   // optional device scalar multiplying alpha (fp8 per-tensor dequantisation)
    bf16_t* ep_aux;           // relu == 2: the pre-activation (bias added) is also stored here (ld = ldc)
    const bf16_t* ep_dgelu;   // multiply the result by gelu'(u), u read from here (GELU backward)
    int acc_c;                // E_F32 (pp engine): C += result instead of C = result
    long long* dbg;           // pp engine: per-block phase timestamps (tools/pp_one.py --trace), or null
    int epi_slack;            // pp engine, plain bf16 epilogues: byte size of C (buffer-store range) with the
                              // store drain deferred under the next item's slices (tuning pp_epi_slack); 0 = off
    int epi_pair;             // pp engine: both wave groups' epilogues in one barrier interval (tuning pp_epi_pair)
};

// GELU (tanh form) through the hardware transcendentals: 0.5 (1 + tanh u) = 1 / (1 + exp(-2u)) = s, one v_exp_f32
// and one v_rcp_f32 (~1 ulp each) instead of the library tanhf (~40 VALU ops with branches, which made the
// GELU epilogue of a K = 768 GEMM cost as much as its MFMAs: GPT-2 fc forward 110 vs 56 us plain).
// exp2 overflows to +inf for u << 0 (s -> 0) and underflows to 0 for u >> 0 (s -> 1): both limits exact.
__device__ __forceinline__ float gelu_sig(float x) {
    const float u = x * (0.7978845608028654f + 0.035677408136300125f * x * x);
    return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.885390081777927f * u));
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_sig(x); }
// d/dx [x s(u)] = s + x * 2 s (1 - s) * u'(x),  u' = 0.79788 (1 + 3 * 0.044715 x^2)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
    const float s = gelu_sig(x);
    return s + 2.f * x * s * (1.f - s) * (0.7978845608028654f + 0.10703222440890037f * x * x);
}

// ---------------------------------------------------------------------------------------------
// LDS image helpers
// ---------------------------------------------------------------------------------------------
// K-major image: [rows][64] bf16, 128-byte rows, 16-byte chunk c of row r stored at chunk c^((r>>1)&7).
__device__ __forceinline__ int kimg_off(int row, int chunk) {   // in bf16 elements
    return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3);
}
// MN-major image: [64 k-rows][W] bf16, W in {64,128,256}; chunk XOR with an even, row-dependent value.
template <int W>
__device__ __forceinline__ int mimg_off(int krow, int chunk) {
    int sw;
    if constexpr (W >= 128) sw = ((krow & 3) | ((krow >> 1) & 4)) << 1;     // 16 (32) chunks / row
    else sw = (((krow >> 1) & 1) | ((krow >> 2) & 2)) << 1;                 // 8 chunks / row
    return krow * W + ((chunk ^ sw) << 3);
}

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ bf16x8_t frag_kmajor(const bf16_t* img, int row, int ks, int lane) {
    const int chunk = ks * 4 + (lane >> 4);
    u16x8_t v = *reinterpret_cast<const u16x8_t*>(img + kimg_off(row, chunk));
    return __builtin_bit_cast(bf16x8_t, v);
}

// Fragment of 16 columns [col0, col0+16) x 32 k (k0 = 32*ks) from an MN-major image via two
// transpose reads: lane 4q+p of each 16-lane group addresses row (k0 + 8g + q [+4]), columns
// col0 + 4p .. +3; lane i receives column col0+i of the four rows.
template <int W>
__device__ __forceinline__ bf16x8_t frag_mnmajor(const bf16_t* img, int col0, int ks, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = col0 + 4 * p;
    const int chunk = col >> 3, within = col & 7;
    const int r0 = ks * 32 + 8 * g + q;
    const bf16_t* p0 = img + mimg_off<W>(r0, chunk) + within;
    const bf16_t* p1 = img + mimg_off<W>(r0 + 4, chunk) + within;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    // Bijective: blocks b, b+8, b+16... (same XCD under round-robin dispatch) get consecutive tiles.
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

typedef __attribute__((address_space(3))) void lds_void;

// compile-time loop: the epilogue body is too large for `#pragma unroll` to be honoured, and a rolled
// fragment loop indexes the accumulator array dynamically, which moves it to scratch memory
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// ping-pong engine entry points (gemm_pp.hip).  amode/bmode/em: AMode/BMode/EMode values.
// pp_supported: operand/shape conditions of the engine; pp_launch returns a hipError_t.
bool pp_supported(const GemmArgs& a, int amode, int bmode, int em, int batch, int splits);
int pp_launch(const GemmArgs& a, int amode, int bmode, int em, hipStream_t st);
int pp_fp8_launch(const GemmArgs& a, int em, hipStream_t st);   // e4m3 operands, K / ld in 2-byte units
int& pp_mode_ref();

}  // namespace pg
