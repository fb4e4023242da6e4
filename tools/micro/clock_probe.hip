// Clock probe (tools only, not the product): the shader clock while a
// benchmark runs.  One wave spins for `us` microseconds of the 100 MHz
// real-time counter and returns how many shader-clock ticks (s_memtime)
// passed meanwhile -> MHz.  tools/clock_ramp.py launches it between renders.
// build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o build/libclockprobe.so tools/micro/clock_probe.hip
#include <hip/hip_runtime.h>

__global__ void clock_probe_kernel(unsigned long long* out, unsigned us) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long ticks = (unsigned long long)us * 100ull;  // 100 MHz
    unsigned long long r = r0;
    while (r - r0 < ticks) r = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;  // shader-clock ticks
        out[1] = r - r0;   // 10 ns ticks
    }
}

extern "C" int clock_probe_launch(unsigned long long* out_device, unsigned us, void* stream) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out_device, us);
    return (int)hipGetLastError();
}
