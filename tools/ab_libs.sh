#!/bin/bash
# A/B timing of built variants on the GPU box: tools/ab_libs.sh ROUNDS name... ("base" = lib/libbwrt.so)
# extra bench args via BENCH_ARGS
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
V=$PWD/bwidman-raytracer_amd/build/variants
R=$1; shift
for r in $(seq $R); do
  for v in "$@"; do
    L=$V/$v/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
    BWRT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$v.log 2>&1
    echo "$v $(grep -o '"ms_per_step[^,]*' gpurun_out/ab_$v.log)"
  done
done
