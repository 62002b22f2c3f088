// MNIST IDX format reader / writer (reference MPI_code/src/mnist/mnist.h:36-138).
//
// Big-endian header: magic = 0x00 0x00 <type> <ndim>, then ndim u32 dims, then raw data.  The reference
// accepts exactly magic 2051 (images, u8, 3 dims) and 2049 (labels, u8, 1 dim); we accept any u8 IDX
// file and report its dims, so both readers' self-tests (mnist.h:88-100) run on synthetic files.
// Normalisation / one-hot / shuffling are done by the Python data layer; the shuffle here is the
// Fisher-Yates of mnist.h:132-138 with a fixed 64-bit seed (xorshift), for the native MLP driver.
#include "runtime.h"

#include <cstdio>
#include <cstring>
#include <vector>

namespace {
uint32_t be32(const unsigned char* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
}

extern "C" {

// Returns number of data bytes (>= 0) or a negative error: -1 open, -2 bad magic, -3 truncated,
// -4 capacity too small (dims still filled).  `dims` must hold 4 ints.
RT_API int pdnn_idx_read(const char* path, uint8_t* out, int64_t cap, int* dims, int* ndim) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    unsigned char hdr[4];
    if (fread(hdr, 1, 4, f) != 4 || hdr[0] != 0 || hdr[1] != 0 || hdr[2] != 0x08 || hdr[3] < 1 || hdr[3] > 4) {
        fclose(f);
        return -2;
    }
    *ndim = hdr[3];
    int64_t total = 1;
    for (int i = 0; i < *ndim; ++i) {
        unsigned char d[4];
        if (fread(d, 1, 4, f) != 4) { fclose(f); return -3; }
        dims[i] = (int)be32(d);
        total *= dims[i];
    }
    if (!out || cap < total) { fclose(f); return -4; }
    const size_t got = fread(out, 1, (size_t)total, f);
    fclose(f);
    return got == (size_t)total ? (int)total : -3;
}

// magic_type: 0x08 (u8).  Writes a big-endian IDX file (used by tests to synthesise MNIST-shaped files).
RT_API int pdnn_idx_write(const char* path, const uint8_t* data, const int* dims, int ndim, int magic_type) {
    FILE* f = fopen(path, "wb");
    if (!f) return -1;
    unsigned char hdr[4] = {0, 0, (unsigned char)magic_type, (unsigned char)ndim};
    fwrite(hdr, 1, 4, f);
    int64_t total = 1;
    for (int i = 0; i < ndim; ++i) {
        unsigned char d[4] = {(unsigned char)(dims[i] >> 24), (unsigned char)(dims[i] >> 16),
                              (unsigned char)(dims[i] >> 8), (unsigned char)dims[i]};
        fwrite(d, 1, 4, f);
        total *= dims[i];
    }
    const size_t w = fwrite(data, 1, (size_t)total, f);
    fclose(f);
    return w == (size_t)total ? 0 : -3;
}

RT_API void pdnn_shuffle_indices(int64_t* idx, int64_t n, uint64_t seed) {
    uint64_t s = seed ? seed : 0x9E3779B97F4A7C15ull;
    for (int64_t i = n - 1; i > 0; --i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const int64_t j = (int64_t)(s % (uint64_t)(i + 1));
        const int64_t t = idx[i]; idx[i] = idx[j]; idx[j] = t;
    }
}
}
