// Direct weight gradient of a 3x3 / stride-1 / pad-1 convolution on MFMA (gfx950):
//   dW[ko][r][s][c] = sum over output pixels p of dy[p][ko] * x[p + (r - 1, s - 1)][c]
// (reference layers: pytorch_code/model_ops/resnet.py:19-21,44-48, every 3x3 conv of the ResNets).
//
// The implicit-GEMM engine (gemm_mfma.hip, A_MNMAJOR x B_IM2COL with split-K atomics) gathers the im2col
// operand from global memory per k-row with two divisions per load, re-reads every input element 9 times
// through L2, and at 2 blocks/CU its one-step register prefetch leaves each K-step waiting on memory:
// 150-350 us per ResNet-50 3x3 layer on the weight-gradient side stream (profiles/resnet50_bs256_timeline_r3b).
//
// Here a block owns one (64 ko x 64 c) chunk pair of the output and a contiguous run of 256-pixel tiles.
// Per tile it stages (a) the dy tile [256 px][64 ko] and (b) the HALO of the tile's input rows (the same
// contiguous NHWC range the forward halo kernel stages, conv3x3.hip) into LDS, then runs the 9 taps as
// shifted reads of the one halo: both operands reach MFMA through the CDNA4 transpose read
// (ds_read_b64_tr_b16), so the pixel dimension -- the reduction -- lands in the fragments' k without any
// transpose pass, and a tap that falls outside the image (padding, or the neighbouring image of a tile that
// straddles two) reads the zero pixel at the end of the halo.  The next tile's dy and halo are fetched into
// registers while the current tile computes (one block of 8 waves per CU, two barriers per tile).
// Accumulation stays in registers across all of the block's tiles (wave w: 16 input channels x 32 output
// channels x 9 taps = 18 fragments); each block writes its partial [64][9][64] once to a workspace slab,
// and a second kernel adds the partials of every chunk pair into dW (the arena's fp32 gradient, +=).
#include "conv_direct.h"

namespace {
using namespace pg;

constexpr int W3_NT = 512;
constexpr int W3_BM = 256;           // pixels per tile
constexpr int W3_HMAX = 512;         // largest supported halo source range (pixels): 8 chunks per thread
constexpr int W3_PS = 64 * 9 * 64 + 64;   // floats per block partial, padded by 256 B: unpadded (147456 B =
                                            // 9 * 16 KB) every partial of an output sat in one HBM channel and the
                                            // reduce crawled (117 us at stage 2)
constexpr int W3_PB = 160;           // bytes per halo pixel (64 channels + 32 B skew): 8 consecutive pixels
                                     // tile the 64 LDS banks, so the transpose reads of 16 pixel rows are 2-way

struct W3Args {
    const bf16_t* x;     // [P][C]
    const bf16_t* dy;    // [P][Ko]
    float* ws;           // [gridDim.x][64 ko][9][64 c] partials, W3_PS floats apart
    int H, W, C, Ko, P;
    FastDiv dW, dH;
    int tiles, cch, G, hrows;
    const float *psc, *psh;   // optional forward prologue: x' = relu(x * psc[c] + psh[c]) (the BN + ReLU that made
                              // the conv's input, applied while staging instead of materialised: fused_resnet a1)
};

// this thread's 8 prologue coefficients (channels c .. c+7), and the prologue on a staged chunk (bn_apply's rounding)
struct W3Pro {
    float sc[8], sh[8];
};
__device__ __forceinline__ void w3_pro_load(const W3Args& a, int c, W3Pro& pr) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { pr.sc[j] = a.psc[c + j]; pr.sh[j] = a.psh[c + j]; }
}
__device__ __forceinline__ u16x8_t w3_pro(const W3Pro& pr, const u16x8_t& v) {
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], pr.sc[j], pr.sh[j]), 0.f);
    return pack8(f);
}

// Halo layout (per tile): the tile's input rows from one above its first to one below its last, each
// image's rows bracketed by an all-zero row above and below, every row padded by a zero pixel left and
// right (pitch WT + 2).  Tap (r, s) of output pixel (y, x) is then halo pixel (hrow(y) + r - 1, x + s) at a
// FIXED offset from the pixel's base for every pixel of the tile: the 9 taps are 9 immediate offsets of one
// address (no per-tap validity, select or swizzle arithmetic; that VALU work was 3x the MFMA time).
//   hrow(gr) = gr - gstart + 2 (img(gr) - img(gstart)) + 1,  gstart = first row - 1 (global row index over
//   the whole batch; img(-1) = -1).
template <int WT, bool FP>
__global__ void __launch_bounds__(W3_NT, 1) conv3x3_wgrad_kernel(W3Args a) {
    constexpr int PITCH = WT + 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const dimg = reinterpret_cast<bf16_t*>(smem);        // [256 px][64 ko], mimg_off<64> swizzle
    char* const halo = smem + W3_BM * 64 * 2;                     // [hrows][PITCH] pixels of W3_PB bytes
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pair = blockIdx.x / a.G, part = blockIdx.x - pair * a.G;
    const int ko0 = (pair / a.cch) * 64, c0 = (pair % a.cch) * 64;
    const int t0 = (int)((long)part * a.tiles / a.G), t1 = (int)((long)(part + 1) * a.tiles / a.G);
    const int hbytes = a.hrows * PITCH * W3_PB;
    [[maybe_unused]] W3Pro pro;
    if constexpr (FP) w3_pro_load(a, c0 + (tid & 7) * 8, pro);       // this thread's halo chunks: i & 7 == tid & 7

    // wave roles: input channels [16 fn, +16), output-channel fragments fmb, fmb + 1 (32 ko), all 9 taps
    const int fn = wave & 3, fmb = (wave >> 2) * 2;
    f32x4_t acc[2][9];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    constexpr int DCH = W3_BM * 8 / W3_NT;      // 4 dy chunks per thread
    constexpr int HCH = W3_HMAX * 8 / W3_NT;    // 8 halo source chunks per thread
    u16x8_t rd[DCH], rh[HCH];
    int nch = 0;                                // source chunks of the tile held in rh
    uint32_t okm = 0;                           // validity of rd (bits 0..3) and rh (bits 4..11): masked at the
                                                // LDS store, so the loads stay in flight under the MFMAs
    int s_gstart = 0, s_istart = 0;             // halo origin of the tile held in the registers

    auto geo = [&](int t, int& p0, int& plast, int& gstart, int& istart) {
        p0 = t * W3_BM;
        plast = min(a.P, p0 + W3_BM) - 1;
        gstart = (int)fdiv((uint32_t)p0, a.dW) - 1;
        istart = gstart < 0 ? -1 : (int)fdiv((uint32_t)gstart, a.dH);
    };
    auto load_regs = [&](int t) {
        int p0, plast, gstart, istart;
        geo(t, p0, plast, gstart, istart);
        s_gstart = gstart;
        s_istart = istart;
#pragma unroll
        for (int j = 0; j < DCH; ++j) {
            const int i = tid + j * W3_NT, row = i >> 3;
            const int p = p0 + row;
            const bool ok = p < a.P;
            rd[j] = *reinterpret_cast<const u16x8_t*>(a.dy + (long)(ok ? p : plast) * a.Ko + ko0 + (i & 7) * 8);
            okm = ok ? (okm | (1u << j)) : (okm & ~(1u << j));
        }
        const int gr1 = (int)fdiv((uint32_t)plast, a.dW);
        nch = (gr1 + 2 - gstart) * WT * 8;      // rows gstart .. gr1 + 1
        const long gp0 = (long)gstart * WT;
#pragma unroll
        for (int j = 0; j < HCH; ++j) {
            const int i = tid + j * W3_NT;
            const long gp = gp0 + (i >> 3);
            const bool ok = i < nch && gp >= 0 && gp < a.P;
            const long gc = gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp);
            rh[j] = *reinterpret_cast<const u16x8_t*>(a.x + gc * a.C + c0 + (i & 7) * 8);
            okm = ok ? (okm | (16u << j)) : (okm & ~(16u << j));
        }
    };
    // zero the whole halo (padding pixels and bracket rows move with every tile), then, after a barrier, the data
    auto zero_halo = [&]() {
        for (int o = tid * 16; o < hbytes; o += W3_NT * 16) *reinterpret_cast<u16x8_t*>(halo + o) = c3_zero8();
    };
    auto store_lds = [&]() {
#pragma unroll
        for (int j = 0; j < DCH; ++j) {
            const int i = tid + j * W3_NT;
            *reinterpret_cast<u16x8_t*>(dimg + mimg_off<64>(i >> 3, i & 7)) = mask16(rd[j], (okm >> j) & 1);
        }
#pragma unroll
        for (int j = 0; j < HCH; ++j) {
            const int i = tid + j * W3_NT;
            if (((okm >> (4 + j)) & 1) != 0) {
                const int gp = s_gstart * WT + (i >> 3);           // >= 0 and < P here
                const int gr = (int)fdiv((uint32_t)gp, a.dW);
                const int xx = gp - gr * WT;
                const int img = (int)fdiv((uint32_t)gr, a.dH);
                const int hrow = gr - s_gstart + 2 * (img - s_istart) + 1;
                u16x8_t hv = rh[j];
                if constexpr (FP) hv = w3_pro(pro, hv);
                *reinterpret_cast<u16x8_t*>(halo + (hrow * PITCH + xx + 1) * W3_PB + (i & 7) * 16) = hv;
            }
        }
    };

    // this lane's transpose-read coordinates: rows k = 32 ks + 8 g + q (+4), input channels 16 fn + 4 pq .. +3
    const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
    const int cbyte = (fn * 16 + 4 * pq) * 2;

    if (t0 < t1) {
        load_regs(t0);
        zero_halo();
    }
    __syncthreads();
    if (t0 < t1) store_lds();
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
        const bool more = t + 1 < t1;
        int p0, plast, gstart, istart;
        geo(t, p0, plast, gstart, istart);
        if (more) load_regs(t + 1);                             // under this tile's MFMAs
#pragma unroll 1
        for (int ks = 0; ks < W3_BM / 32; ++ks) {
            bf16x8_t af[2];
#pragma unroll
            for (int f = 0; f < 2; ++f) af[f] = frag_mnmajor<64>(dimg, (fmb + f) * 16, ks, lane);
            // byte address of tap (0, 0) for the two pixels of this lane's transpose reads; pixels past P read
            // real (finite) halo data against an all-zero dy row
            int base[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int p = min(p0 + ks * 32 + 8 * g + q + 4 * h, plast);
                const int gr = (int)fdiv((uint32_t)p, a.dW);
                const int xx = p - gr * WT;
                const int img = (int)fdiv((uint32_t)gr, a.dH);
                const int hrow = gr - gstart + 2 * (img - istart) + 1;
                base[h] = ((hrow - 1) * PITCH + xx) * W3_PB + cbyte;
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int off = ((tap / 3) * PITCH + tap % 3) * W3_PB;
                const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(halo + base[0] + off));
                const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(halo + base[1] + off));
                typedef __attribute__((ext_vector_type(8))) short s16x8;
                const s16x8 xv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                const bf16x8_t xf = __builtin_bit_cast(bf16x8_t, xv);
#pragma unroll
                for (int f = 0; f < 2; ++f)
                    acc[f][tap] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f], xf, acc[f][tap], 0, 0, 0);
            }
        }
        __syncthreads();                          // every wave is done reading this tile's images
        if (more) {
            zero_halo();
            __syncthreads();
            store_lds();
            __syncthreads();
        }
    }
    // partial of this block: lane holds dW[ko = 16 (fmb + f) + 4 g + j][tap][c = 16 fn + (lane & 15)]
    float* ws = a.ws + (long)blockIdx.x * W3_PS;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ko = (fmb + f) * 16 + 4 * g + j;
                ws[(ko * 9 + tap) * 64 + fn * 16 + (lane & 15)] = acc[f][tap][j];
            }
}

// ---------------------------------------------------------------------------------------------------------------
// fp8 variant (BASELINE config 5): the same block structure, the operands quantised while they are staged (dy with
// the data gradient's e5m2 scale, x with the forward's e4m3 scale: both were just rolled to the exact |max| of these
// very tensors by the fp8 halo conv that consumed them) and reduced 128 pixels per v_mfma_scale_f32_16x16x128_f8f6f4.
// Both operands reach MFMA through ds_read_b64_tr_b8 (dev/probes/tr8_probe.hip: lane i of a 16-lane group addresses
// row i / 2, bytes 8 (i & 1) .. +7, and receives column i of the 8 rows): four reads give a lane its 32 pixels of one
// channel.  Images: dy [256 px][64 ko] bytes with the 16-byte chunks XOR-swizzled by w8_swz (the 16 pixel rows
// a 32-lane half reads fall on 16 distinct 4-bank groups); halo pixels of 64 channel bytes + 16 skew (W8_PB).
constexpr int W8_PB = 80;

__device__ __forceinline__ int w8_swz(int r) { return ((r >> 2) & 1) | (((r >> 5) & 1) << 1); }
__device__ __forceinline__ int w8_doff(int r, int c16) { return r * 64 + ((c16 ^ w8_swz(r)) << 4); }

// 8 floats -> 8 fp8 bytes (FMT 0: e4m3fn / 448, 1: e5m2 / 57344), saturating
template <int FMT>
__device__ __forceinline__ uint2 w8_cvt(const u16x8_t& v, float s) {
    constexpr float MX = FMT ? 57344.f : 448.f;
    float f[8];
    unpack8(v, f);
    int w[2];
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        const float c0 = fminf(fmaxf(f[4 * d] * s, -MX), MX), c1 = fminf(fmaxf(f[4 * d + 1] * s, -MX), MX);
        const float c2 = fminf(fmaxf(f[4 * d + 2] * s, -MX), MX), c3 = fminf(fmaxf(f[4 * d + 3] * s, -MX), MX);
        int x = 0;
        if constexpr (FMT) {
            x = __builtin_amdgcn_cvt_pk_bf8_f32(c0, c1, x, false);
            x = __builtin_amdgcn_cvt_pk_bf8_f32(c2, c3, x, true);
        } else {
            x = __builtin_amdgcn_cvt_pk_fp8_f32(c0, c1, x, false);
            x = __builtin_amdgcn_cvt_pk_fp8_f32(c2, c3, x, true);
        }
        w[d] = x;
    }
    return make_uint2((uint32_t)w[0], (uint32_t)w[1]);
}

typedef __attribute__((ext_vector_type(2))) int w8v2i;
typedef __attribute__((ext_vector_type(8))) int w8v8i;
typedef __attribute__((address_space(3))) w8v2i lds_w8v2i;

struct W8Scale {
    const float *sx, *sdy;     // quantisation scales of x (e4m3) and dy (e5m2)
    const float *ix, *idy;     // their inverses (the partials are dequantised by ix * idy)
};

template <int WT, bool FP>
__global__ void __launch_bounds__(W3_NT, 1) conv3x3_wgrad8_kernel(W3Args a, W8Scale q) {
    constexpr int PITCH = WT + 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const dimg = smem;                                      // [256 px][64 ko] e5m2, w8_doff
    char* const halo = smem + W3_BM * 64;                         // [hrows][PITCH] pixels of W8_PB bytes
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pair = blockIdx.x / a.G, part = blockIdx.x - pair * a.G;
    const int ko0 = (pair / a.cch) * 64, c0 = (pair % a.cch) * 64;
    const int t0 = (int)((long)part * a.tiles / a.G), t1 = (int)((long)(part + 1) * a.tiles / a.G);
    const int hbytes = a.hrows * PITCH * W8_PB;
    const float sx = q.sx[0], sdy = q.sdy[0];
    [[maybe_unused]] W3Pro pro;
    if constexpr (FP) w3_pro_load(a, c0 + (tid & 7) * 8, pro);

    const int fn = wave & 3, fmb = (wave >> 2) * 2;
    f32x4_t acc[2][9];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    constexpr int DCH = W3_BM * 8 / W3_NT;
    constexpr int HCH = W3_HMAX * 8 / W3_NT;
    u16x8_t rd[DCH], rh[HCH];
    int nch = 0;
    uint32_t okm = 0;
    int s_gstart = 0, s_istart = 0;

    auto geo = [&](int t, int& p0, int& plast, int& gstart, int& istart) {
        p0 = t * W3_BM;
        plast = min(a.P, p0 + W3_BM) - 1;
        gstart = (int)fdiv((uint32_t)p0, a.dW) - 1;
        istart = gstart < 0 ? -1 : (int)fdiv((uint32_t)gstart, a.dH);
    };
    auto load_regs = [&](int t) {
        int p0, plast, gstart, istart;
        geo(t, p0, plast, gstart, istart);
        s_gstart = gstart;
        s_istart = istart;
#pragma unroll
        for (int j = 0; j < DCH; ++j) {
            const int i = tid + j * W3_NT, row = i >> 3;
            const int p = p0 + row;
            const bool ok = p < a.P;
            rd[j] = *reinterpret_cast<const u16x8_t*>(a.dy + (long)(ok ? p : plast) * a.Ko + ko0 + (i & 7) * 8);
            okm = ok ? (okm | (1u << j)) : (okm & ~(1u << j));
        }
        const int gr1 = (int)fdiv((uint32_t)plast, a.dW);
        nch = (gr1 + 2 - gstart) * WT * 8;
        const long gp0 = (long)gstart * WT;
#pragma unroll
        for (int j = 0; j < HCH; ++j) {
            const int i = tid + j * W3_NT;
            const long gp = gp0 + (i >> 3);
            const bool ok = i < nch && gp >= 0 && gp < a.P;
            const long gc = gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp);
            rh[j] = *reinterpret_cast<const u16x8_t*>(a.x + gc * a.C + c0 + (i & 7) * 8);
            okm = ok ? (okm | (16u << j)) : (okm & ~(16u << j));
        }
    };
    auto zero_halo = [&]() {
        for (int o = tid * 16; o < hbytes; o += W3_NT * 16) *reinterpret_cast<u16x8_t*>(halo + o) = c3_zero8();
    };
    auto store_lds = [&]() {
#pragma unroll
        for (int j = 0; j < DCH; ++j) {
            const int i = tid + j * W3_NT, row = i >> 3, qq = i & 7;
            const uint2 v = w8_cvt<1>(rd[j], sdy);
            const uint32_t m = ((okm >> j) & 1) ? 0xFFFFFFFFu : 0u;
            *reinterpret_cast<uint2*>(dimg + w8_doff(row, qq >> 1) + 8 * (qq & 1)) = make_uint2(v.x & m, v.y & m);
        }
#pragma unroll
        for (int j = 0; j < HCH; ++j) {
            const int i = tid + j * W3_NT;
            if (((okm >> (4 + j)) & 1) != 0) {
                const int gp = s_gstart * WT + (i >> 3);
                const int gr = (int)fdiv((uint32_t)gp, a.dW);
                const int xx = gp - gr * WT;
                const int img = (int)fdiv((uint32_t)gr, a.dH);
                const int hrow = gr - s_gstart + 2 * (img - s_istart) + 1;
                u16x8_t hv = rh[j];
                if constexpr (FP) hv = w3_pro(pro, hv);
                *reinterpret_cast<uint2*>(halo + (hrow * PITCH + xx + 1) * W8_PB + (i & 7) * 8) = w8_cvt<0>(hv, sx);
            }
        }
    };

    const int g = lane >> 4, li = lane & 15, lr = li >> 1, lh = 8 * (li & 1);

    if (t0 < t1) {
        load_regs(t0);
        zero_halo();
    }
    __syncthreads();
    if (t0 < t1) store_lds();
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
        const bool more = t + 1 < t1;
        int p0, plast, gstart, istart;
        geo(t, p0, plast, gstart, istart);
        if (more) load_regs(t + 1);
#pragma unroll 1
        for (int ks = 0; ks < W3_BM / 128; ++ks) {
            // dy^T fragments: ko column 16 (fmb + f) + li, pixels 128 ks + 32 g + 0..31 (four 8-row transposed reads)
            w8v8i af[2];
#pragma unroll
            for (int f = 0; f < 2; ++f)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = ks * 128 + 32 * g + 8 * j + lr;
                    const w8v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_w8v2i*)(dimg + w8_doff(r, fmb + f) + lh));
                    af[f][2 * j] = v[0];
                    af[f][2 * j + 1] = v[1];
                }
            // halo byte address of tap (0, 0) for the pixel this lane addresses in each 8-pixel read (past P: real
            // halo bytes against all-zero dy rows)
            int base[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int p = min(p0 + ks * 128 + 32 * g + 8 * j + lr, plast);
                const int gr = (int)fdiv((uint32_t)p, a.dW);
                const int xx = p - gr * WT;
                const int img = (int)fdiv((uint32_t)gr, a.dH);
                const int hrow = gr - gstart + 2 * (img - istart) + 1;
                base[j] = ((hrow - 1) * PITCH + xx) * W8_PB + 16 * fn + lh;
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int off = ((tap / 3) * PITCH + tap % 3) * W8_PB;
                w8v8i xf;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const w8v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_w8v2i*)(halo + base[j] + off));
                    xf[2 * j] = v[0];
                    xf[2 * j + 1] = v[1];
                }
#pragma unroll
                for (int f = 0; f < 2; ++f)
                    acc[f][tap] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[f], xf, acc[f][tap], 1, 0, 0,
                                                                                   0x7f7f7f7f, 0, 0x7f7f7f7f);
            }
        }
        __syncthreads();
        if (more) {
            zero_halo();
            __syncthreads();
            store_lds();
            __syncthreads();
        }
    }
    const float dq = q.ix[0] * q.idy[0];
    float* ws = a.ws + (long)blockIdx.x * W3_PS;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ko = (fmb + f) * 16 + 4 * g + j;
                ws[(ko * 9 + tap) * 64 + fn * 16 + (lane & 15)] = acc[f][tap][j] * dq;
            }
}

// ---------------------------------------------------------------------------------------------------------------
// Stride-2 weight gradient (the 3x3 / stride-2 / pad-1 conv2 of a ResNet stage-transition Bottleneck; reference:
// pytorch_code/model_ops/resnet.py:39-56):
//   dW[ko][r][s][c] = sum over half-resolution pixels p = (n, i, j) of dy[p][ko] * x[n][2i + r - 1][2j + s - 1][c].
// Tap (r, s) reads the input's parity plane (a, b) = (r != 1, s != 1) at half-resolution offset (dr, ds), dr = -1 for
// r = 0 and 0 for r = 1, 2 (likewise ds).  Every plane is a half-resolution image, so the stride-1 kernel's padded halo
// layout holds it unchanged and the plane's taps are immediate offsets (dr + 1, ds + 1) of one address.  A tile's dy is
// staged once and its four plane halos follow one after the other (stage = (tile, plane), 1 / 2 / 2 / 4 taps), each
// gathered from NHWC x with stride-2 pixel addresses into registers under the previous stage's MFMAs.  FP: the BN + ReLU
// of the layer below applied while staging (a1 never materialised).  a.H / a.W: the half-resolution extent.
template <int WT, bool FP>
__global__ void __launch_bounds__(W3_NT, 1) conv3x3s2_wgrad_kernel(W3Args a) {
    constexpr int PITCH = WT + 2;
    constexpr int XW = 2 * WT;                // input width
    extern __shared__ __attribute__((aligned(16))) char smem[];
    bf16_t* const dimg = reinterpret_cast<bf16_t*>(smem);
    char* const halo = smem + W3_BM * 64 * 2;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int pair = blockIdx.x / a.G, part = blockIdx.x - pair * a.G;
    const int ko0 = (pair / a.cch) * 64, c0 = (pair % a.cch) * 64;
    const int t0 = (int)((long)part * a.tiles / a.G), t1 = (int)((long)(part + 1) * a.tiles / a.G);
    const int hbytes = a.hrows * PITCH * W3_PB;
    [[maybe_unused]] W3Pro pro;
    if constexpr (FP) w3_pro_load(a, c0 + (tid & 7) * 8, pro);

    const int fn = wave & 3, fmb = (wave >> 2) * 2;
    f32x4_t acc[2][9];
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[f][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    constexpr int DCH = W3_BM * 8 / W3_NT;
    constexpr int HCH = W3_HMAX * 8 / W3_NT;
    u16x8_t rd[DCH], rh[HCH];
    uint32_t okm = 0;
    int s_gstart = 0, s_istart = 0;

    auto geo = [&](int t, int& p0, int& plast, int& gstart, int& istart) {
        p0 = t * W3_BM;
        plast = min(a.P, p0 + W3_BM) - 1;
        gstart = (int)fdiv((uint32_t)p0, a.dW) - 1;
        istart = gstart < 0 ? -1 : (int)fdiv((uint32_t)gstart, a.dH);
    };
    // registers <- (tile t's dy if with_dy) + plane (pa, pb) of its input rows gstart .. gr1 (half resolution)
    auto load_regs = [&](int t, int pa, int pb, bool with_dy) {
        int p0, plast, gstart, istart;
        geo(t, p0, plast, gstart, istart);
        s_gstart = gstart;
        s_istart = istart;
        if (with_dy) {
#pragma unroll
            for (int j = 0; j < DCH; ++j) {
                const int i = tid + j * W3_NT, row = i >> 3;
                const int p = p0 + row;
                const bool ok = p < a.P;
                rd[j] = *reinterpret_cast<const u16x8_t*>(a.dy + (long)(ok ? p : plast) * a.Ko + ko0 + (i & 7) * 8);
                okm = ok ? (okm | (1u << j)) : (okm & ~(1u << j));
            }
        }
        const int gr1 = (int)fdiv((uint32_t)plast, a.dW);
        const int nch = (gr1 + 1 - gstart) * WT * 8;        // rows gstart .. gr1 (the taps reach one row up only)
        const long gp0 = (long)gstart * WT;
#pragma unroll
        for (int j = 0; j < HCH; ++j) {
            const int i = tid + j * W3_NT;
            const long gp = gp0 + (i >> 3);
            const bool ok = i < nch && gp >= 0 && gp < a.P;
            const int gc = (int)(gp < 0 ? 0 : (gp >= a.P ? a.P - 1 : gp));
            const int gr = (int)fdiv((uint32_t)gc, a.dW);
            const long xp = (long)(2 * gr + pa) * XW + 2 * (gc - gr * WT) + pb;
            rh[j] = *reinterpret_cast<const u16x8_t*>(a.x + xp * a.C + c0 + (i & 7) * 8);
            okm = ok ? (okm | (16u << j)) : (okm & ~(16u << j));
        }
    };
    auto zero_halo = [&]() {
        for (int o = tid * 16; o < hbytes; o += W3_NT * 16) *reinterpret_cast<u16x8_t*>(halo + o) = c3_zero8();
    };
    auto store_lds = [&](bool with_dy) {
        if (with_dy) {
#pragma unroll
            for (int j = 0; j < DCH; ++j) {
                const int i = tid + j * W3_NT;
                *reinterpret_cast<u16x8_t*>(dimg + mimg_off<64>(i >> 3, i & 7)) = mask16(rd[j], (okm >> j) & 1);
            }
        }
#pragma unroll
        for (int j = 0; j < HCH; ++j) {
            const int i = tid + j * W3_NT;
            if (((okm >> (4 + j)) & 1) != 0) {
                const int gp = s_gstart * WT + (i >> 3);
                const int gr = (int)fdiv((uint32_t)gp, a.dW);
                const int xx = gp - gr * WT;
                const int img = (int)fdiv((uint32_t)gr, a.dH);
                const int hrow = gr - s_gstart + 2 * (img - s_istart) + 1;
                u16x8_t hv = rh[j];
                if constexpr (FP) hv = w3_pro(pro, hv);
                *reinterpret_cast<u16x8_t*>(halo + (hrow * PITCH + xx + 1) * W3_PB + (i & 7) * 16) = hv;
            }
        }
    };

    const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
    const int cbyte = (fn * 16 + 4 * pq) * 2;
    const int s0 = t0 * 4, s1 = t1 * 4;

    if (s0 < s1) {
        load_regs(t0, 0, 0, true);
        zero_halo();
    }
    __syncthreads();
    if (s0 < s1) store_lds(true);
    __syncthreads();
    for (int st = s0; st < s1; ++st) {
        const int t = st >> 2, plane = st & 3;
        const bool more = st + 1 < s1;
        int p0, plast, gstart, istart;
        geo(t, p0, plast, gstart, istart);
        if (more) {
            const int nx = (st + 1) & 3;
            load_regs((st + 1) >> 2, nx >> 1, nx & 1, nx == 0);          // under this stage's MFMAs
        }
        // plane (pa, pb): taps r in {1} (pa = 0) or {0, 2}, s likewise; compile-time per plane (static accumulators)
        static_for<0, 4>([&](auto PL) {
            constexpr int PA = decltype(PL)::value >> 1, PB = decltype(PL)::value & 1;
            if (plane != decltype(PL)::value) return;
#pragma unroll 1
            for (int ks = 0; ks < W3_BM / 32; ++ks) {
                bf16x8_t af[2];
#pragma unroll
                for (int f = 0; f < 2; ++f) af[f] = frag_mnmajor<64>(dimg, (fmb + f) * 16, ks, lane);
                int base[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int p = min(p0 + ks * 32 + 8 * g + q + 4 * h, plast);
                    const int gr = (int)fdiv((uint32_t)p, a.dW);
                    const int xx = p - gr * WT;
                    const int img = (int)fdiv((uint32_t)gr, a.dH);
                    const int hrow = gr - gstart + 2 * (img - istart) + 1;
                    base[h] = ((hrow - 1) * PITCH + xx) * W3_PB + cbyte;
                }
                static_for<0, (1 + PA) * (1 + PB)>([&](auto K) {
                    constexpr int k = decltype(K)::value;
                    constexpr int kr = PB ? (k >> 1) : k, kc = PB ? (k & 1) : 0;
                    constexpr int r = PA ? 2 * kr : 1, s = PB ? 2 * kc : 1;
                    constexpr int off = ((r == 0 ? 0 : 1) * PITCH + (s == 0 ? 0 : 1)) * W3_PB;
                    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(halo + base[0] + off));
                    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(halo + base[1] + off));
                    typedef __attribute__((ext_vector_type(8))) short s16x8;
                    const s16x8 xv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    const bf16x8_t xf = __builtin_bit_cast(bf16x8_t, xv);
#pragma unroll
                    for (int f = 0; f < 2; ++f)
                        acc[f][3 * r + s] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f], xf, acc[f][3 * r + s], 0, 0, 0);
                });
            }
        });
        __syncthreads();                          // every wave is done reading this stage's images
        if (more) {
            zero_halo();
            __syncthreads();
            store_lds(((st + 1) & 3) == 0);
            __syncthreads();
        }
    }
    float* ws = a.ws + (long)blockIdx.x * W3_PS;
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ko = (fmb + f) * 16 + 4 * g + j;
                ws[(ko * 9 + tap) * 64 + fn * 16 + (lane & 15)] = acc[f][tap][j];
            }
}

int w3_hrows(int H, int W);
int w8_smem(int H, int W);

// dW[ko][tap][c] += sum over the G partials of chunk pair (ko / 64, c / 64).  A block covers OUT = 256 / PG
// consecutive float4 outputs with PG partial groups (PG ~ G / 8, so every thread sums ~8 partials with all its
// loads in flight); the groups are combined through LDS.  (One thread per output summing all G partials was a
// G/8-deep latency chain: 92 us at stage 1, G = 256.)
template <int PG>
__global__ void __launch_bounds__(256) conv3x3_wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                                                    int Ko, int C, int cch, int G) {
    constexpr int OUT = 256 / PG;
    __shared__ float4 red[PG][OUT];
    const int o = threadIdx.x % OUT, pg = threadIdx.x / OUT;
    const long total = (long)Ko * 9 * (C / 4);
    const long i = (long)blockIdx.x * OUT + o;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    int c = 0, tap = 0, ko = 0;
    if (i < total) {
        c = (int)(i % (C / 4)) * 4;
        const long r = i / (C / 4);
        tap = (int)(r % 9);
        ko = (int)(r / 9);
        const int pair = (ko >> 6) * cch + (c >> 6);
        const float* src = ws + (long)pair * G * W3_PS + (ko & 63) * 576 + tap * 64 + (c & 63);
        constexpr long BS = W3_PS;
        int b = pg;
        for (; b + 7 * PG < G; b += 8 * PG) {
            float4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const float4*>(src + (b + PG * j) * BS);
#pragma unroll
            for (int j = 0; j < 8; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
        }
        for (; b < G; b += PG) {
            const float4 v = *reinterpret_cast<const float4*>(src + b * BS);
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    if constexpr (PG > 1) {
        red[pg][o] = s;
        __syncthreads();
    }
    if (pg == 0 && i < total) {
#pragma unroll
        for (int k = 1; k < PG; ++k) { const float4 v = red[k][o]; s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
        float4* d = reinterpret_cast<float4*>(dw + ((long)ko * 9 + tap) * C + c);
        const float4 cur = *d;
        *d = make_float4(cur.x + s.x, cur.y + s.y, cur.z + s.z, cur.w + s.w);
    }
}

// halo rows of the padded layout: source rows R = ceil((BM - 1 + W - 1) / W) + 3, plus a zero row above and
// below every image they touch, plus one
int w3_hrows(int H, int W) {
    const int R = (W3_BM - 1 + W - 1) / W + 1 + 2;
    const int imgs = (R + H - 1) / H + 1;
    return R + 2 * imgs + 1;
}
int w3_smem(int H, int W) { return W3_BM * 64 * 2 + w3_hrows(H, W) * (W + 2) * W3_PB; }
int w8_smem(int H, int W) { return W3_BM * 64 + w3_hrows(H, W) * (W + 2) * W8_PB; }

void w3_plan(int P, int C, int Ko, int& tiles, int& cch, int& G) {
    tiles = (P + W3_BM - 1) / W3_BM;
    cch = C / 64;
    const int pairs = (Ko / 64) * cch;
    // ~128 blocks in total (half the CUs): the kernel runs on the side stream beside the data-gradient chain, and a
    // smaller grid leaves more of the chip to it (ResNet-50 same box: 128 vs 256 blocks +0.6..+0.7%, 64 +0.1..+0.3%
    // more, 512 -1%; gpurun_out/r4_61-62)
    G = (128 + pairs - 1) / pairs;
    if (G > tiles) G = tiles;
    if (G < 1) G = 1;
}

// the 160 KB dynamic-LDS opt-in, once per kernel instantiation (whichever variant a call picks)
void w3_attr(const void* fn) {
    static const void* done[32] = {};
    for (int i = 0; i < 32; ++i) {
        if (done[i] == fn) return;
        if (!done[i]) {
            (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            done[i] = fn;
            return;
        }
    }
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

FastDiv w3_fdiv(uint32_t d) {
    FastDiv f;
    f.d = d ? d : 1;
    uint32_t l = 0;
    while ((1ull << l) < f.d) ++l;
    f.s = l;
    f.m = (uint32_t)((((1ull << l) - f.d) << 32) / f.d + 1);
    return f;
}
}  // namespace

// Whether the direct kernel takes this 3x3 / stride-1 / pad-1 weight gradient (image widths 7/14/28/56: the
// ResNet stages; the tap offsets are compile-time immediates).
PDNN_API int pdnn_conv3x3_wgrad_supported(int Nimg, int H, int W, int C, int Ko) {
    if (C % 64 || Ko % 64 || C < 64 || Ko < 64 || H < 1) return 0;
    if (W != 7 && W != 14 && W != 28 && W != 56) return 0;
    if ((long)Nimg * H * W >= (1L << 31) / 2) return 0;
    if (((W3_BM - 1 + W - 1) / W + 3) * W > W3_HMAX) return 0;
    return w3_smem(H, W) <= 160 * 1024 ? 1 : 0;
}

// floats of workspace pdnn_conv3x3_wgrad needs
PDNN_API int pdnn_conv3x3_wgrad_ws(int Nimg, int H, int W, int C, int Ko) {
    int tiles, cch, G;
    w3_plan(Nimg * H * W, C, Ko, tiles, cch, G);
    return (Ko / 64) * cch * G * W3_PS;
}

// fp8 weight gradient (conv3x3_wgrad8_kernel): x quantised to e4m3 with sx[0], dy to e5m2 with sdy[0], the partials
// dequantised by ix[0] * idy[0]; same shapes, workspace and reduce as pdnn_conv3x3_wgrad.
PDNN_API int pdnn_conv3x3_wgrad_fp8(const bf16_t* x, const bf16_t* dy, float* dw, int Nimg, int H, int W, int C, int Ko,
                                    float* ws, const float* sx, const float* sdy, const float* ix, const float* idy,
                                    const float* pro_sc, const float* pro_sh, hipStream_t st) {
    if (!pdnn_conv3x3_wgrad_supported(Nimg, H, W, C, Ko) || !ws || !sx || !sdy || !ix || !idy)
        return (int)hipErrorInvalidValue;
    W3Args a{};
    a.x = x; a.dy = dy; a.ws = ws;
    a.H = H; a.W = W; a.C = C; a.Ko = Ko; a.P = Nimg * H * W;
    a.dW = w3_fdiv(W); a.dH = w3_fdiv(H);
    w3_plan(a.P, C, Ko, a.tiles, a.cch, a.G);
    a.hrows = w3_hrows(H, W);
    if (!pro_sc != !pro_sh) return (int)hipErrorInvalidValue;
    a.psc = pro_sc; a.psh = pro_sh;
    const bool fp = pro_sc != nullptr;
    const W8Scale q{sx, sdy, ix, idy};
    const int sm = w8_smem(H, W);
    const int grid = (Ko / 64) * a.cch * a.G;
#define W8_GO(WT, F)                                                                                             \
    do {                                                                                                         \
        w3_attr((const void*)conv3x3_wgrad8_kernel<WT, F>);                                                      \
        hipLaunchKernelGGL((conv3x3_wgrad8_kernel<WT, F>), dim3(grid), dim3(W3_NT), sm, st, a, q);                \
    } while (0)
#define W8_W(WT) do { if (fp) W8_GO(WT, true); else W8_GO(WT, false); } while (0)
    if (W == 56) W8_W(56); else if (W == 28) W8_W(28); else if (W == 14) W8_W(14); else W8_W(7);
#undef W8_W
#undef W8_GO
    const int e = (int)hipGetLastError();
    if (e) return e;
    const long outs = (long)Ko * 9 * (C / 4);
#define W3_R(PG) hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel<PG>, dim3((unsigned)cdiv(outs, 256 / PG)), dim3(256), 0, st, \
                                    (const float*)ws, dw, Ko, C, a.cch, a.G)
    if (a.G >= 256) W3_R(32);
    else if (a.G >= 128) W3_R(16);
    else if (a.G >= 64) W3_R(8);
    else if (a.G >= 32) W3_R(4);
    else if (a.G >= 16) W3_R(2);
    else W3_R(1);
#undef W3_R
    PDNN_LAUNCH_RET;
}

// dw [Ko][3][3][C] fp32 += weight gradient of y = conv3x3(x, w) (stride 1, pad 1) given dy [P][Ko]
// pro_sc / pro_sh (optional, both or neither): x is the pre-activation t of relu(t * pro_sc + pro_sh), applied as the
// halo is staged
PDNN_API int pdnn_conv3x3_wgrad(const bf16_t* x, const bf16_t* dy, float* dw, int Nimg, int H, int W, int C, int Ko,
                                float* ws, const float* pro_sc, const float* pro_sh, hipStream_t st) {
    if (!pdnn_conv3x3_wgrad_supported(Nimg, H, W, C, Ko) || !ws) return (int)hipErrorInvalidValue;
    W3Args a{};
    a.x = x; a.dy = dy; a.ws = ws;
    a.H = H; a.W = W; a.C = C; a.Ko = Ko; a.P = Nimg * H * W;
    a.dW = w3_fdiv(W); a.dH = w3_fdiv(H);
    w3_plan(a.P, C, Ko, a.tiles, a.cch, a.G);
    a.hrows = w3_hrows(H, W);
    if (!pro_sc != !pro_sh) return (int)hipErrorInvalidValue;
    a.psc = pro_sc; a.psh = pro_sh;
    const bool fp = pro_sc != nullptr;
    const int sm = w3_smem(H, W);
    const int grid = (Ko / 64) * a.cch * a.G;
#define W3_GO(WT, F)                                                                                             \
    do {                                                                                                         \
        w3_attr((const void*)conv3x3_wgrad_kernel<WT, F>);                                                       \
        hipLaunchKernelGGL((conv3x3_wgrad_kernel<WT, F>), dim3(grid), dim3(W3_NT), sm, st, a);                   \
    } while (0)
#define W3_W(WT) do { if (fp) W3_GO(WT, true); else W3_GO(WT, false); } while (0)
    if (W == 56) W3_W(56); else if (W == 28) W3_W(28); else if (W == 14) W3_W(14); else W3_W(7);
#undef W3_W
#undef W3_GO
    const int e = (int)hipGetLastError();
    if (e) return e;
    const long outs = (long)Ko * 9 * (C / 4);
#define W3_R(PG) hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel<PG>, dim3((unsigned)cdiv(outs, 256 / PG)), dim3(256), 0, st, \
                                    (const float*)ws, dw, Ko, C, a.cch, a.G)
    if (a.G >= 256) W3_R(32);
    else if (a.G >= 128) W3_R(16);
    else if (a.G >= 64) W3_R(8);
    else if (a.G >= 32) W3_R(4);
    else if (a.G >= 16) W3_R(2);
    else W3_R(1);
#undef W3_R
    PDNN_LAUNCH_RET;
}

// Whether the stride-2 direct weight gradient takes this conv (input H x W even, half-resolution width 7 / 14 / 28,
// channel multiples of 64, the plane halo within the stride-1 kernel's limits).
PDNN_API int pdnn_conv3x3s2_wgrad_supported(int Nimg, int H, int W, int C, int Ko) {
    if (H % 2 || W % 2) return 0;
    const int Wo = W / 2;
    if (Wo != 7 && Wo != 14 && Wo != 28) return 0;
    return pdnn_conv3x3_wgrad_supported(Nimg, H / 2, Wo, C, Ko);
}

PDNN_API int pdnn_conv3x3s2_wgrad_ws(int Nimg, int H, int W, int C, int Ko) {
    return pdnn_conv3x3_wgrad_ws(Nimg, H / 2, W / 2, C, Ko);
}

// dw [Ko][3][3][C] fp32 += weight gradient of y = conv3x3/s2/p1(x [Nimg][H][W][C]) given dy [Nimg][H/2][W/2][Ko];
// pro_sc / pro_sh: x is the pre-activation of relu(x * sc + sh), applied as the planes are staged.
PDNN_API int pdnn_conv3x3s2_wgrad(const bf16_t* x, const bf16_t* dy, float* dw, int Nimg, int H, int W, int C, int Ko,
                                  float* ws, const float* pro_sc, const float* pro_sh, hipStream_t st) {
    if (!pdnn_conv3x3s2_wgrad_supported(Nimg, H, W, C, Ko) || !ws || (!pro_sc != !pro_sh))
        return (int)hipErrorInvalidValue;
    const int Ho = H / 2, Wo = W / 2;
    W3Args a{};
    a.x = x; a.dy = dy; a.ws = ws;
    a.H = Ho; a.W = Wo; a.C = C; a.Ko = Ko; a.P = Nimg * Ho * Wo;
    a.dW = w3_fdiv(Wo); a.dH = w3_fdiv(Ho);
    w3_plan(a.P, C, Ko, a.tiles, a.cch, a.G);
    a.hrows = w3_hrows(Ho, Wo);
    a.psc = pro_sc; a.psh = pro_sh;
    const bool fp = pro_sc != nullptr;
    const int sm = w3_smem(Ho, Wo);
    const int grid = (Ko / 64) * a.cch * a.G;
#define W3S_GO(WT, F)                                                                                            \
    do {                                                                                                         \
        w3_attr((const void*)conv3x3s2_wgrad_kernel<WT, F>);                                                     \
        hipLaunchKernelGGL((conv3x3s2_wgrad_kernel<WT, F>), dim3(grid), dim3(W3_NT), sm, st, a);                 \
    } while (0)
#define W3S_W(WT) do { if (fp) W3S_GO(WT, true); else W3S_GO(WT, false); } while (0)
    if (Wo == 28) W3S_W(28); else if (Wo == 14) W3S_W(14); else W3S_W(7);
#undef W3S_W
#undef W3S_GO
    const int e = (int)hipGetLastError();
    if (e) return e;
    const long outs = (long)Ko * 9 * (C / 4);
#define W3_R(PG) hipLaunchKernelGGL(conv3x3_wgrad_reduce_kernel<PG>, dim3((unsigned)cdiv(outs, 256 / PG)), dim3(256), 0, st, \
                                    (const float*)ws, dw, Ko, C, a.cch, a.G)
    if (a.G >= 256) W3_R(32);
    else if (a.G >= 128) W3_R(16);
    else if (a.G >= 64) W3_R(8);
    else if (a.G >= 32) W3_R(4);
    else if (a.G >= 16) W3_R(2);
    else W3_R(1);
#undef W3_R
    PDNN_LAUNCH_RET;
}
