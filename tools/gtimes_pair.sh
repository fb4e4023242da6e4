#!/bin/bash
# Group spans of the c3 shards under the launch policy (pair kernel at 1/8 and
# 1/16, 256-lane sorted groups at 1/4): -DRT_GTIMES variant
# (tools/variants.sh gtimes -DRT_GTIMES)
export BWRT_TUNING=1
set -o pipefail
for g in 4 8 16; do
  for p in 1 0; do
    echo "pair=$p"
    BWRT_PAIR=$p BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/gtimes/libbwrt.so timeout -k 10 120 python tools/gtimes_run.py c3 $g 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
