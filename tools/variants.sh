#!/bin/bash
# Build libbwrt.so variants for A/B timing: tools/variants.sh name "EXTRA FLAGS" ...
# -> bwidman-raytracer_amd/build/variants/<name>/libbwrt.so  (SRC=dir: another source tree, e.g. a git export)
set -e
cd "$(dirname "$0")/../bwidman-raytracer_amd"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=build/variants/$name; mkdir -p $out
  /opt/rocm/bin/hipcc -O1 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-unroll-loops -fvisibility=hidden ${TUNE:--DRT_WAVES_PER_EU=6 -DRT_SORTED_BLOCK=256} $flags \
     -c -o $out/k.o ${SRC:-csrc}/rt_kernels.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-unroll-loops -fvisibility=hidden ${TUNE:--DRT_WAVES_PER_EU=6 -DRT_SORTED_BLOCK=256} $flags \
     ${BVHFLAGS:--URT_WAVES_PER_EU -DRT_WAVES_PER_EU=4} -c -o $out/kb.o ${SRC:-csrc}/rt_kernels_bvh.hip
  /opt/rocm/bin/hipcc -O1 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden ${TUNE:--DRT_WAVES_PER_EU=6 -DRT_SORTED_BLOCK=256} $flags \
     -x hip -c -o $out/c.o ${SRC:-csrc}/rt_context.cpp
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -x hip --cuda-host-only -march=x86-64-v3 -ffp-contract=off -fvisibility=hidden $flags \
     -c -o $out/cpu.o ${SRC:-csrc}/rt_cpu.cpp
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-rpath,/opt/rocm/lib -o $out/libbwrt.so $out/k.o $out/kb.o $out/c.o $out/cpu.o
  /opt/rocm/bin/hipcc -O1 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-unroll-loops $flags --cuda-device-only -c \
     -Rpass-analysis=kernel-resource-usage -o /dev/null ${SRC:-csrc}/rt_kernels.hip 2>&1 | grep -A2 "rt_render_kernelILi256ELb1" | grep -E "VGPRs:|SGPRs" | sed "s/^/$name: /" || true
done
