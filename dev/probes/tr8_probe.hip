// Lane semantics of ds_read_b64_tr_b8 (gfx950): LDS holds a 16 x 16 byte block, byte (r, c) = 16 r + c.
// Hypothesis: lane i of a 16-lane group supplies the address of row i / 2, bytes 8 (i & 1) .. +7, and receives
// column i of the 8 rows (row q in byte q).  Prints what each lane of group 0 receives.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(2))) int v2i;
typedef __attribute__((address_space(3))) v2i lds_v2i;
__global__ void k(unsigned long long* o) {
    __shared__ __attribute__((aligned(16))) unsigned char s[256];
    for (int i = threadIdx.x; i < 256; i += 64) s[i] = (unsigned char)i;
    __syncthreads();
    const int i = threadIdx.x & 15;
    const int row = i >> 1, col = 8 * (i & 1);
    v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_v2i*)(s + row * 16 + col));
    o[threadIdx.x] = (unsigned long long)(unsigned)r[0] | ((unsigned long long)(unsigned)r[1] << 32);
}
int main() {
    unsigned long long* d;
    unsigned long long h[64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int l = 0; l < 16; ++l) {
        printf("lane %2d:", l);
        for (int b = 0; b < 8; ++b) printf(" %3d", (int)((h[l] >> (8 * b)) & 0xff));
        printf("\n");
    }
    return 0;
}
