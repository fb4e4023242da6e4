#!/bin/bash
# Shard-sweep kernel times for several built variants on the GPU box:
# tools/sweep_libs.sh "STRIDES" name... ("base" = lib/libbwrt.so); extra args via SWEEP_ARGS
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
V=$PWD/bwidman-raytracer_amd/build/variants
S=$1; shift
for v in "$@"; do
  L=$V/$v/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
  BWRT_LIB=$L timeout -k 10 120 python tools/shard_sweep.py --strides $S --blocks 0 $SWEEP_ARGS 2>&1 | grep median | sed "s/^/$v: /" || exit 1
done
