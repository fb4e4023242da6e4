#!/bin/bash
# A/B of launch-order feedback variants on c3 row shards: tools/ab_order.sh name... ("base" = lib/libbwrt.so)
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
for v in "$@"; do
  L=$PWD/bwidman-raytracer_amd/build/variants/$v/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
  BWRT_LIB=$L timeout -k 10 150 python tools/shard_sweep.py --strides ${STRIDES:-1,2,4,8} --blocks 0 --reps ${REPS:-20} > gpurun_out/ab_order_$v.log 2>&1 || exit 1
  echo "$v: $(grep -o 'stride [0-9]*: median [0-9.]*' gpurun_out/ab_order_$v.log | tr '\n' ' ')"
done
