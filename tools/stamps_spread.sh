#!/bin/bash
# RT_STAMPS phase counters of the sorted kernel on c3 row shards: 1/4 (128-lane
# groups, no spread) and 1/8, 1/16 (spread groups, split closest hits).  Build
# the stamps variant first: tools/variants.sh stamps -DRT_STAMPS
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
mkdir -p gpurun_out/stamps_spread
for g in ${STRIDES:-4 8 16}; do
  BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/stamps/libbwrt.so timeout -k 10 120 python tools/stamps_run.py $g > gpurun_out/stamps_spread/st$g.log 2>&1 || { tail -5 gpurun_out/stamps_spread/st$g.log; exit 1; }
  echo "stride=$g"; grep stamps gpurun_out/stamps_spread/st$g.log
done
# group spans (-DRT_GTIMES variant: tools/variants.sh gtimes -DRT_GTIMES)
for g in ${GSTRIDES:-4 8 16}; do
  echo "gtimes stride=$g"
  BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/gtimes/libbwrt.so timeout -k 10 120 python tools/gtimes_run.py c3 $g 2>&1 | grep -v amdgpu.ids || exit 1
done
