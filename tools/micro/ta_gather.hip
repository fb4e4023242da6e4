// Micro-benchmark (tools only, not the product): cost of per-lane gathers
// from an L2-resident buffer on MI355X, by load width and by how many lanes
// of a wave share a cache line — does the walk's bound (TA busy, config 5)
// scale with lanes, bytes or distinct lines?
// build: hipcc --offload-arch=gfx950 -O3 -o build/ta_gather tools/micro/ta_gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int W>  // dwords per lane: 1, 2, 4
__global__ void __launch_bounds__(256) gather(const unsigned* __restrict__ buf, unsigned mask_lines, int share,
                                              int iters, unsigned* out) {
    const unsigned lane = threadIdx.x & 63;
    unsigned x = blockIdx.x * 2654435761u + (threadIdx.x / 64) * 40503u;  // per-wave seed
    unsigned acc = 0;
    for (int i = 0; i < iters; i++) {
        x = x * 1664525u + 1013904223u;
        // lanes of a wave in groups of `share` read the same 16-byte slot of
        // one 128-byte line; groups read unrelated lines
        const unsigned grp = lane / share;
        const unsigned line = ((x >> 8) + grp * 2246822519u) & mask_lines;
        const unsigned* p = buf + line * 32 + (lane % share % 8) * 4 * 0;
        if (W == 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(p);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (W == 2) {
            const uint2 v = *reinterpret_cast<const uint2*>(p);
            acc += v.x ^ v.y;
        } else {
            acc += *p;
        }
        x ^= acc & 1;  // dependent chain: the next address waits for the load
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t lines = 1 << 15;  // 32 K lines x 128 B = 4 MB: L2-resident (4 MB per XCD)
    unsigned *buf, *out;
    hipMalloc(&buf, lines * 128);
    hipMalloc(&out, 4);
    hipMemset(buf, 1, lines * 128);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grid = 256 * 16, iters = 2000;
    // footprint: 4 MB (L2-resident, every distinct line an L1 miss) and
    // 16 KB (128 lines: L1-resident after the first touch, L1 hits)
    for (size_t fp : {lines, (size_t)128})
    for (int w : {1, 2, 4})
        for (int share : {1, 2, 4, 8, 16, 64}) {
            if (fp != lines && w != 4) continue;
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (w == 4) hipLaunchKernelGGL(gather<4>, dim3(grid), dim3(256), 0, 0, buf, (unsigned)(fp - 1), share, iters, out);
                if (w == 2) hipLaunchKernelGGL(gather<2>, dim3(grid), dim3(256), 0, 0, buf, (unsigned)(fp - 1), share, iters, out);
                if (w == 1) hipLaunchKernelGGL(gather<1>, dim3(grid), dim3(256), 0, 0, buf, (unsigned)(fp - 1), share, iters, out);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double winst = (double)grid * 4 * iters;  // wave-level load instructions
                if (rep) printf("footprint %7zu B  dwords/lane %d  lanes per line %2d: %.3f ms  %.2f G wave-loads/s  %.2f cycles per wave-load per CU\n",
                                fp * 128, w, share, ms, winst / ms / 1e6, ms * 1e-3 * 2.4e9 * 256 / winst);
            }
        }
    return 0;
}
