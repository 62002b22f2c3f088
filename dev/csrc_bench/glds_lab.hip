// Standalone A/B bench of glds GEMM main-loop schedules (plain C = A . B^T, both operands K-major bf16,
// bf16 output), to pick the schedule for csrc/kernels/gemm_glds.h without perturbing the library build
// (cdna_hip_programming.md §5.4 rules 19 and 24: variants compared in one process, interleaved rounds).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 csrc/bench/glds_lab.hip -o build/glds_lab && build/glds_lab
//
// Variants (256-row tiles, BK = 64, 8 waves, XCD-aware tile order):
//   v0  2 LDS stages; every next-tile glds issued at the top of the K-step; vmcnt(0) + __syncthreads
//       at its end (the library's schedule)
//   v1  2 stages; glds issue spread one wave-instruction at a time between the MFMA groups of the K-step
//       (pinned with sched_barrier), s_setprio(1) around the MFMA groups
//   v2  3 LDS stages (BN <= 128): one K-step's glds kept in flight across a raw s_barrier with a counted
//       vmcnt; issue at the top
//   v3  v2 with the spread issue of v1
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(8))) unsigned short u16x8_t;
typedef __attribute__((address_space(3))) void lds_void;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1); } } while (0)

constexpr int BM = 256, BK = 64, NTH = 512;

__device__ __forceinline__ int kimg_off(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ bf16x8_t frag(const bf16_t* img, int row, int ks, int lane) {
    const int chunk = ks * 4 + (lane >> 4);
    return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const u16x8_t*>(img + kimg_off(row, chunk)));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / 8, r = nwg % 8, x = bid % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

template <int N>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
// (target builtins wrapped in __device__ helpers: used directly in a __global__ template body they make the
// host pass drop the kernel stub)
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
template <int P>
__device__ __forceinline__ void setprio() { __builtin_amdgcn_s_setprio(P); }
__device__ __forceinline__ void raw_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// K-major rows loader: ROWS rows x 64 k per stage, NI wave-instructions per wave (8 rows each)
template <int ROWS>
struct Ld {
    static constexpr int NI = ROWS / 8 / 8;
    const bf16_t* base[NI];
    int k;
    __device__ void init(const bf16_t* p, long ld, int rows_total, int row0, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int row = row0 + 8 * (wave * NI + i) + (lane >> 3);
            base[i] = p + (long)min(row, rows_total - 1) * ld;
        }
        k = 0;
    }
    __device__ __forceinline__ void one(int i, bf16_t* img, int wave, int lane) {
        const int rr = 8 * (wave * NI + i) + (lane >> 3);
        const int ch = ((lane & 7) ^ ((rr >> 1) & 7)) * 8;
        __builtin_amdgcn_global_load_lds(base[i] + k + ch, (lds_void*)(img + (wave * NI + i) * 512), 16, 0, 0);
    }
    __device__ __forceinline__ void issue(bf16_t* img, int wave, int lane) {
#pragma unroll
        for (int i = 0; i < NI; ++i) one(i, img, wave, lane);
        k += BK;
    }
};

template <int BN> struct Waves;
template <> struct Waves<256> { static constexpr int WM = 2, WN = 4; };
template <> struct Waves<128> { static constexpr int WM = 4, WN = 2; };

template <int BN, int VAR>
constexpr int lab_smem() { return ((VAR >= 2) ? 3 : 2) * (BM + BN) * BK * 2; }

template <int BN, int VAR>
__global__ void __launch_bounds__(NTH) lab_gemm(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                 bf16_t* __restrict__ C, int M, int N, int K) {
    constexpr int WM = Waves<BN>::WM, WN = Waves<BN>::WN;
    constexpr int WTM = BM / WM, WTN = BN / WN, FM = WTM / 16, FN = WTN / 16;
    constexpr int IMA = BM * BK, IMB = BN * BK, STG = IMA + IMB;
    constexpr int NSTG = VAR >= 2 ? 3 : 2;
    constexpr bool SPREAD = VAR == 1 || VAR == 3;
    using LA = Ld<BM>;
    using LB = Ld<BN>;
    constexpr int IPS = LA::NI + LB::NI;          // glds wave-instructions per stage
    constexpr int SLOTS = 2 * FM;                 // MFMA groups per K-step
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const sb = reinterpret_cast<bf16_t*>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int tiles_n = (N + BN - 1) / BN, ntiles = ((M + BM - 1) / BM) * tiles_n;
    const int t = xcd_remap(blockIdx.x, ntiles);
    const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
    const int kt1 = K / BK;
    LA la;
    LB lb;
    la.init(A, K, M, m0, wave, lane);
    lb.init(B, K, N, n0, wave, lane);
    f32x4_t acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // one K-step on image `cur`, issuing the next stage into `nxt` (nullptr: none)
    auto step = [&](const bf16_t* cur, bf16_t* nxt) {
        const bf16_t* A_ = cur;
        const bf16_t* B_ = cur + IMA;
        if (!SPREAD && nxt) { la.issue(nxt, wave, lane); lb.issue(nxt + IMA, wave, lane); }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8_t bfr[FN];
#pragma unroll
            for (int f = 0; f < FN; ++f) bfr[f] = frag(B_, wn * WTN + f * 16 + (lane & 15), ks, lane);
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
                const bf16x8_t af = frag(A_, wm * WTM + fm * 16 + (lane & 15), ks, lane);
                if constexpr (SPREAD) {
                    const int slot = ks * FM + fm;
                    if (nxt) {
#pragma unroll
                        for (int j = 0; j < IPS; ++j) {
                            if ((j * SLOTS) / IPS == slot) {
                                sched_fence();
                                if (j < LA::NI) la.one(j, nxt, wave, lane);
                                else lb.one(j - LA::NI, nxt + IMA, wave, lane);
                                sched_fence();
                            }
                        }
                    }
                    setprio<1>();
                }
#pragma unroll
                for (int fn = 0; fn < FN; ++fn)
                    acc[fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[fn], af, acc[fm][fn], 0, 0, 0);
                if constexpr (SPREAD) setprio<0>();
            }
        }
        if (SPREAD && nxt) { la.k += BK; lb.k += BK; }
    };

    if constexpr (NSTG == 2) {
        la.issue(sb, wave, lane);
        lb.issue(sb + IMA, wave, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int cur = 0;
        for (int kt = 0; kt < kt1; ++kt) {
            step(sb + cur * STG, kt + 1 < kt1 ? sb + (cur ^ 1) * STG : nullptr);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            cur ^= 1;
        }
    } else {
        la.issue(sb, wave, lane);
        lb.issue(sb + IMA, wave, lane);
        if (kt1 > 1) { la.issue(sb + STG, wave, lane); lb.issue(sb + STG + IMA, wave, lane); }
        int buf = 0;
        for (int kt = 0; kt < kt1; ++kt) {
            if (kt + 1 < kt1) vm_wait<IPS>(); else vm_wait<0>();
            raw_barrier();
            const int nb = buf == 0 ? 2 : buf - 1;
            step(sb + buf * STG, kt + 2 < kt1 ? sb + nb * STG : nullptr);
            buf = buf == 2 ? 0 : buf + 1;
        }
    }
    const int lm = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int fm = 0; fm < FM; ++fm) {
        const int m = m0 + wm * WTM + fm * 16 + lm;
        if (m >= M) continue;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            const int n = n0 + wn * WTN + fn * 16 + 4 * lg;
            if (n + 4 > N) continue;
            __bf16 b0 = (__bf16)acc[fm][fn][0], b1 = (__bf16)acc[fm][fn][1];
            __bf16 b2 = (__bf16)acc[fm][fn][2], b3 = (__bf16)acc[fm][fn][3];
            uint2 pk;
            pk.x = (uint32_t)__builtin_bit_cast(uint16_t, b0) | ((uint32_t)__builtin_bit_cast(uint16_t, b1) << 16);
            pk.y = (uint32_t)__builtin_bit_cast(uint16_t, b2) | ((uint32_t)__builtin_bit_cast(uint16_t, b3) << 16);
            *reinterpret_cast<uint2*>(C + (long)m * N + n) = pk;
        }
    }
}

// explicit instantiations (the host pass otherwise omits the stubs of the variants whose bodies call the
// scheduling builtins)
#define LAB_INST(BN, V) template __global__ void lab_gemm<BN, V>(const bf16_t* __restrict__, \
    const bf16_t* __restrict__, bf16_t* __restrict__, int, int, int);
LAB_INST(256, 0) LAB_INST(256, 1) LAB_INST(128, 0) LAB_INST(128, 1) LAB_INST(128, 2) LAB_INST(128, 3)

__global__ void ref_gemm(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
    const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
    if (n >= N) return;
    float s = 0.f;
    for (int k = 0; k < K; ++k)
        s += __uint_as_float((uint32_t)A[(long)m * K + k] << 16) * __uint_as_float((uint32_t)B[(long)n * K + k] << 16);
    C[(long)m * N + n] = s;
}

template <int BN, int VAR>
float run(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int iters) {
    constexpr int SM = lab_smem<BN, VAR>();
    static bool attr = false;
    if (!attr) {
        attr = true;
        CK(hipFuncSetAttribute((const void*)lab_gemm<BN, VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, SM));
    }
    const int tiles = (int)(((M + BM - 1) / BM) * ((N + BN - 1) / BN));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL((lab_gemm<BN, VAR>), dim3(tiles), dim3(NTH), SM, 0, A, B, C, M, N, K);
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL((lab_gemm<BN, VAR>), dim3(tiles), dim3(NTH), SM, 0, A, B, C, M, N, K);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / iters;
}

static float bf2f_h(bf16_t v) {
    uint32_t u = (uint32_t)v << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

template <int BN, int VAR>
bool check(const bf16_t* A, const bf16_t* B, bf16_t* C, const float* R, int M, int N, int K, const char* tag) {
    run<BN, VAR>(A, B, C, M, N, K, 1);
    CK(hipDeviceSynchronize());
    std::vector<bf16_t> h((size_t)M * N);
    std::vector<float> r((size_t)M * N);
    CK(hipMemcpy(h.data(), C, h.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(r.data(), R, r.size() * 4, hipMemcpyDeviceToHost));
    double md = 0, mx = 0;
    for (size_t i = 0; i < h.size(); ++i) {
        md = std::max(md, (double)std::fabs(bf2f_h(h[i]) - r[i]));
        mx = std::max(mx, (double)std::fabs(r[i]));
    }
    const bool ok = md / mx < 1e-2;
    printf("{\"check\": \"%s\", \"rel_err\": %.3e, \"ok\": %s}\n", tag, md / mx, ok ? "true" : "false");
    fflush(stdout);
    return ok;
}

struct Shape { const char* name; int M, N, K; };

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const Shape shapes[] = {
        {"sq8192", 8192, 8192, 8192}, {"sq4096", 4096, 4096, 4096}, {"gpt2_qkv", 8192, 2304, 768},
        {"gpt2_fc", 8192, 3072, 768}, {"gpt2_fc2", 8192, 768, 3072}, {"gpt2_head", 8192, 50304, 768},
        {"r50_l3_1x1", 50176, 1024, 256}, {"gpt2_proj", 8192, 768, 768},
    };
    size_t maxA = 0, maxB = 0, maxC = 0;
    for (auto& s : shapes) {
        maxA = std::max(maxA, (size_t)s.M * s.K);
        maxB = std::max(maxB, (size_t)s.N * s.K);
        maxC = std::max(maxC, (size_t)s.M * s.N);
    }
    bf16_t *A, *B, *C;
    CK(hipMalloc(&A, maxA * 2));
    CK(hipMalloc(&B, maxB * 2));
    CK(hipMalloc(&C, maxC * 2));
    {
        std::mt19937 g(1);
        std::uniform_real_distribution<float> u(-1.f, 1.f);
        std::vector<bf16_t> h(std::max(maxA, maxB));
        for (auto& v : h) {
            const float f = u(g);
            uint32_t x;
            memcpy(&x, &f, 4);
            v = (bf16_t)((x + 0x7fff + ((x >> 16) & 1)) >> 16);
        }
        CK(hipMemcpy(A, h.data(), maxA * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(B, h.data(), maxB * 2, hipMemcpyHostToDevice));
    }
    bool ok = true;
    {   // correctness on a ragged shape (M, N not multiples of the tile)
        const int M = 1000, N = 1000, K = 1024;
        float* R;
        CK(hipMalloc(&R, (size_t)M * N * 4));
        hipLaunchKernelGGL(ref_gemm, dim3((N + 255) / 256, M), dim3(256), 0, 0, A, B, R, M, N, K);
        CK(hipDeviceSynchronize());
        ok &= check<256, 0>(A, B, C, R, M, N, K, "bn256_v0");
        ok &= check<256, 1>(A, B, C, R, M, N, K, "bn256_v1");
        ok &= check<128, 0>(A, B, C, R, M, N, K, "bn128_v0");
        ok &= check<128, 1>(A, B, C, R, M, N, K, "bn128_v1");
        ok &= check<128, 2>(A, B, C, R, M, N, K, "bn128_v2");
        ok &= check<128, 3>(A, B, C, R, M, N, K, "bn128_v3");
        CK(hipFree(R));
    }
    if (!ok) return 1;
    for (auto& s : shapes) {
        const double fl = 2.0 * s.M * s.N * s.K;
        const int it = fl > 1e12 ? 5 : 20;
        std::vector<float> t[6];
        for (int r = 0; r < rounds; ++r) {
            t[0].push_back(run<256, 0>(A, B, C, s.M, s.N, s.K, it));
            t[1].push_back(run<256, 1>(A, B, C, s.M, s.N, s.K, it));
            t[2].push_back(run<128, 0>(A, B, C, s.M, s.N, s.K, it));
            t[3].push_back(run<128, 1>(A, B, C, s.M, s.N, s.K, it));
            t[4].push_back(run<128, 2>(A, B, C, s.M, s.N, s.K, it));
            t[5].push_back(run<128, 3>(A, B, C, s.M, s.N, s.K, it));
        }
        const char* names[6] = {"bn256_v0", "bn256_v1", "bn128_v0", "bn128_v1", "bn128_v2", "bn128_v3"};
        printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d", s.name, s.M, s.N, s.K);
        for (int v = 0; v < 6; ++v) {
            std::sort(t[v].begin(), t[v].end());
            printf(", \"%s\": %.0f", names[v], fl / (t[v][t[v].size() / 2] * 1e-3) / 1e12);
        }
        printf("}\n");
        fflush(stdout);
    }
    return 0;
}
