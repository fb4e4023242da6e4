// Exhaustive check of the gfx950 hardware v_sqrt_f32 / v_rcp_f32 against the
// correctly rounded sqrtf / 1.0f/x (HIP's default fp32 lowering) over every
// float bit pattern.  Prints per-class mismatch counts and the first few
// mismatches.  Build: hipcc -O2 --offload-arch=gfx950 -o build/hwmath tools/hw_math_exhaustive.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

struct Counts {
    unsigned long long sqrt_bad[4];  // [denormal, normal, zero/inf, nan]
    unsigned long long rcp_bad[4];
    unsigned first_sqrt[8], first_rcp[8];
};

__device__ int cls(float x) {
    if (x != x) return 3;
    const float ax = fabsf(x);
    if (ax == 0.0f || ax == INFINITY) return 2;
    if (ax < 1.17549435e-38f) return 0;
    return 1;
}

__global__ void check(unsigned long long base, Counts* c) {
    const unsigned long long i = base + (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned bits = (unsigned)i;
    const float x = __uint_as_float(bits);
    const float hs = __builtin_amdgcn_sqrtf(x);
    const float rs = sqrtf(x);
    const float hr = __builtin_amdgcn_rcpf(x);
    const float rr = 1.0f / x;
    const int k = cls(x);
    const bool sbad = __float_as_uint(hs) != __float_as_uint(rs) && !(hs != hs && rs != rs);
    const bool rbad = __float_as_uint(hr) != __float_as_uint(rr) && !(hr != hr && rr != rr);
    if (sbad) {
        unsigned long long n = atomicAdd(&c->sqrt_bad[k], 1ull);
        if (k == 1 && n < 8) c->first_sqrt[n] = bits;
    }
    if (rbad) {
        unsigned long long n = atomicAdd(&c->rcp_bad[k], 1ull);
        if (k == 1 && n < 8) c->first_rcp[n] = bits;
    }
}

int main() {
    Counts* d;
    hipMalloc(&d, sizeof(Counts));
    hipMemset(d, 0, sizeof(Counts));
    const unsigned long long total = 1ull << 32, chunk = 1ull << 28;
    for (unsigned long long b = 0; b < total; b += chunk) check<<<chunk / 256, 256>>>(b, d);
    Counts h;
    hipMemcpy(&h, d, sizeof(Counts), hipMemcpyDeviceToHost);
    const char* nm[4] = {"denormal", "normal", "zero/inf", "nan"};
    for (int k = 0; k < 4; k++)
        printf("%-9s sqrt mismatches %llu  rcp mismatches %llu\n", nm[k], h.sqrt_bad[k], h.rcp_bad[k]);
    for (int j = 0; j < 8 && j < (int)h.sqrt_bad[1]; j++) {
        float x; memcpy(&x, &h.first_sqrt[j], 4);
        printf("sqrt bad: %08x %.9g\n", h.first_sqrt[j], x);
    }
    for (int j = 0; j < 8 && j < (int)h.rcp_bad[1]; j++) {
        float x; memcpy(&x, &h.first_rcp[j], 4);
        printf("rcp bad: %08x %.9g\n", h.first_rcp[j], x);
    }
    return 0;
}
