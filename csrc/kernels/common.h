// Shared device helpers for the CDNA4 (gfx950) kernel library.
//
// Conventions used by every kernel in this directory:
//  * bf16 tensors are passed as raw `uint16_t*` (bit pattern), converted with the helpers below;
//    the float->bf16 conversion is a plain `__bf16` cast, which hipcc lowers to
//    `v_cvt_pk_bf16_f32` (round-to-nearest-even, NaN preserving).
//  * Every launcher is `extern "C" int pdnn_<name>(..., hipStream_t)` returning the hipError_t of the
//    launch, so the Python side can raise loudly.  No launcher allocates or synchronises: they are
//    safe inside hipGraph capture (cdna_hip_programming.md Guideline 9).
//  * Wavefront = 64 lanes.  Block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define PDNN_API extern "C" __attribute__((visibility("default")))
#define PDNN_LAUNCH_RET return (int)hipGetLastError()

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;   // MFMA A/B operand (16x16x32 / 32x32x16)
typedef __attribute__((ext_vector_type(4))) float f32x4_t;     // 16x16 accumulator fragment
typedef __attribute__((ext_vector_type(16))) float f32x16_t;   // 32x32 accumulator fragment
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8_t;
typedef __attribute__((ext_vector_type(4))) unsigned short u16x4_t;
typedef __attribute__((ext_vector_type(2))) unsigned short u16x2_t;

constexpr int kWave = 64;

// BatchNorm statistics "slabs" are STAT_BINS row pairs [bin][sum | second][C] that producers ADD into with
// fp32 atomics (no-return global_atomic_add_f32; partial row r goes to bin r % STAT_BINS), not one stored row
// pair per tile: the finalize then reads 64 rows instead of up to 12544 (ResNet-50 stage 1) and zeroes them
// again for the next producer (batchnorm.hip bn_slab_final_kernel).  Summation order varies run to run in the
// last fp32 bits.
constexpr int STAT_BINS = 64;
__device__ __forceinline__ float* stat_row(float* slab, long row, int C) {
    return slab + (long)(2 * (row & (STAT_BINS - 1))) * C;
}
__device__ __forceinline__ void stat_add(float* p, float v) { atomicAdd(p, v); }
// The statistics of one 16-column MFMA fragment in ONE atomic instruction: after row16_sum every lane of a 16-lane
// row holds the 4 columns' sums (s) and second sums (q) of its column group lg = lane >> 4; lane lm = lane & 15 < 4
// adds s[lm] to column 4 lg + lm of the s row, lane 4 <= lm < 8 adds q[lm - 4] to the q row (ps / pq: this lane's
// column group, column 4 lg), 32 lanes on two 64-byte lines.  It replaces eight 4-lane atomics (one per (j, s|q)):
// ResNet-50's A-stationary 1x1 forwards spent 23-57 us per call on them (gpurun_out/r6_21).  `ok` (per lane):
// this lane's column exists; qx (optional) transforms the q value of column j before the add.
__device__ __forceinline__ float sel4(const float (&v)[4], int j) {
    return j == 0 ? v[0] : (j == 1 ? v[1] : (j == 2 ? v[2] : v[3]));
}
__device__ __forceinline__ void stat_add_frag(float* ps, float* pq, int lane, const float (&s)[4], const float (&q)[4],
                                              bool ok) {
    const int lm = lane & 15, j = lm & 3;
    if (lm < 8 && ok) stat_add(lm < 4 ? ps + j : pq + j, lm < 4 ? sel4(s, j) : sel4(q, j));
}

__device__ __forceinline__ float bf2f(bf16_t v) {
    return __uint_as_float(((uint32_t)v) << 16);
}
__device__ __forceinline__ bf16_t f2bf(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(bf16_t, b);
}
// two floats -> packed bf16 pair (lo = a) in ONE v_cvt_pk_bf16_f32 (the scalar form above takes two conversions, a
// shift and an or per pair)
typedef float f32x2_cv_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_cv_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk2bf(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_cv_t{a, b}, bf16x2_cv_t));
}

template <typename T> struct Ld;
template <> struct Ld<float> {
    static __device__ __forceinline__ float get(const float* p, long i) { return p[i]; }
    static __device__ __forceinline__ void put(float* p, long i, float v) { p[i] = v; }
};
template <> struct Ld<bf16_t> {
    static __device__ __forceinline__ float get(const bf16_t* p, long i) { return bf2f(p[i]); }
    static __device__ __forceinline__ void put(bf16_t* p, long i, float v) { p[i] = f2bf(v); }
};

// DPP lane moves (VALU, no LDS round trip like ds_bpermute-based __shfl_xor)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Sum over each 16-lane row; every lane of the row receives the row total.
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0xB1>(v);     // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);     // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);    // row_half_mirror: quads 0<->1, 2<->3
    v += dpp_f<0x140>(v);    // row_mirror: half-rows swap
    return v;
}

__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    v = fmaxf(v, dpp_f<0x140>(v));
    return v;
}
__device__ __forceinline__ float readlane_f(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
// Whole-wave reductions (all 64 lanes active): DPP within 16-lane rows, then the 4 row results via
// v_readlane (scalar) -- no LDS traffic.
__device__ __forceinline__ float wave_sum(float v) {
    v = row16_sum(v);
    return (readlane_f(v, 0) + readlane_f(v, 16)) + (readlane_f(v, 32) + readlane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
    v = row16_max(v);
    return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}

// Block-wide sum for blockDim.x == NT (multiple of 64).  `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l == 0) red[w] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    __syncthreads();
    return t;
}

// Unpack 8 bf16 (16 bytes) to floats and back.
__device__ __forceinline__ void unpack8(const u16x8_t& v, float* f) {
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = bf2f(v[i]);
}
__device__ __forceinline__ u16x8_t pack8(const float* f) {
    u16x8_t v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = f2bf(f[i]);
    return v;
}

__host__ __device__ constexpr inline long cdiv(long a, long b) { return (a + b - 1) / b; }

// Grid size for grid-stride memory-bound kernels: <= 8 blocks/CU * 256 CUs (Guideline 11).
inline unsigned stream_grid(long work_items, int per_block) {
    long g = (work_items + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > 512) g = 512;   // 2 blocks per CU walking the grid-stride loop: GPT-2 +0.4%, ResNet-50 flat vs 2048 (r4_68)
    return (unsigned)g;
}
