#!/bin/bash
# Group-span distribution of the c3 shards with the tail off / on (-DRT_GTIMES
# variant: tools/variants.sh gtimes -DRT_GTIMES)
export BWRT_TUNING=1
set -o pipefail
for g in 8 16; do
  for t in 0 4 16; do
    echo "tail=$t"
    BWRT_TAIL=$t BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/gtimes/libbwrt.so timeout -k 10 120 python tools/gtimes_run.py c3 $g 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
