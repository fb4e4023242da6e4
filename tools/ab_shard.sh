#!/bin/bash
# A/B of built variants on one row shard: tools/ab_shard.sh CONFIG STRIDE name... ("base" = lib/libbwrt.so)
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
C=$1; S=$2; shift 2
for v in "$@"; do
  L=$PWD/bwidman-raytracer_amd/build/variants/$v/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
  echo "$v $(BWRT_LIB=$L timeout -k 10 120 python tools/shard_sweep.py --config $C --strides $S --blocks 0 --reps ${REPS:-5} 2>&1 | tail -1)" || exit 1
done
