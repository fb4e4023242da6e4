#!/bin/bash
# Pair-kernel build options: the working library vs build/variants/{o3,pw8}
# (-O3 for the kernel TU; an 8-wave occupancy target), small shards and the
# full frame.  usage: [ROUNDS=2] [VARS="main o3 pw8"] bash tools/ab_pairopt.sh
export BWRT_TUNING=1
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARS:-main o3 pw8}; do
    if [ $v = main ]; then L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so; else L=$V/$v/libbwrt.so; fi
    for c in c3:1,8,16 c2:8; do
      BWRT_LIB=$L timeout -k 10 150 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 2>&1 | grep stride | sed "s/^/$v /" || exit 1
    done
  done
done
