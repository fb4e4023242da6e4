// Exhaustive check of bwidman-raytracer_amd/csrc/rt_sqrt.h against HIP's
// correctly rounded lowering over every fp32 bit pattern (NaN == NaN):
// sqrt_cr(x) == sqrtf(x), rcp_cr(x) == 1.0f / x,
// inv_length_cr(x) == 1.0f / sqrtf(x).
// Build: hipcc -O2 --offload-arch=gfx950 -Ibwidman-raytracer_amd/csrc -o build/sqrtx tools/sqrt_exhaustive.hip
// Exit status 0 iff there is no mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>

#include "rt_sqrt.h"

__device__ __forceinline__ bool differ(float a, float b) {
    return __float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b);
}

__global__ void check(unsigned long long base, unsigned long long* bad, unsigned* first) {
    const unsigned bits = (unsigned)(base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const int k = differ(sqrt_cr(x), sqrtf(x)) ? 0 : differ(rcp_cr(x), 1.0f / x) ? 1
                : differ(inv_length_cr(x), 1.0f / sqrtf(x)) ? 2 : -1;
    if (k >= 0) {
        const unsigned long long n = atomicAdd(&bad[k], 1ull);
        if (n < 8) first[8 * k + n] = bits;
    }
}

int main() {
    unsigned long long* bad;
    unsigned* first;
    if (hipMalloc(&bad, 24) != hipSuccess || hipMalloc(&first, 96) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 24);
    const unsigned long long total = 1ull << 32, chunk = 1ull << 28;
    for (unsigned long long b = 0; b < total; b += chunk) check<<<chunk / 256, 256>>>(b, bad, first);
    unsigned long long h[3] = {};
    unsigned f[24] = {};
    if (hipMemcpy(h, bad, 24, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    (void)hipMemcpy(f, first, 96, hipMemcpyDeviceToHost);
    const char* nm[3] = {"sqrt_cr vs sqrtf", "rcp_cr vs 1/x", "inv_length_cr vs 1/sqrtf"};
    for (int k = 0; k < 3; k++) {
        printf("%s over 2^32 inputs: %llu mismatches\n", nm[k], h[k]);
        for (int j = 0; j < 8 && j < (int)h[k]; j++) printf("  mismatch at %08x\n", f[8 * k + j]);
    }
    return h[0] + h[1] + h[2] == 0 ? 0 : 1;
}
