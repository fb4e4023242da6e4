#!/bin/bash
# A/B of two libbwrt.so builds on one GPU box: alternating config benches
# (kernel event average) and c3 row-shard sweeps.
# usage: A=label:path B=label:path [ROUNDS=3] [CONFIGS="c3 c4"] [STRIDES=1,4,8,16] bash tools/ab_pair.sh
# (path "base" = bwidman-raytracer_amd/lib/libbwrt.so, otherwise a variant name
# under bwidman-raytracer_amd/build/variants)
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
OUT=gpurun_out/ab_pair; mkdir -p $OUT
lib() { [ "$1" = base ] && echo $PWD/bwidman-raytracer_amd/lib/libbwrt.so || echo $V/$1/libbwrt.so; }
for r in $(seq ${ROUNDS:-3}); do
  for spec in "$A" "$B"; do
    IFS=: read -r label var <<< "$spec"; L=$(lib $var)
    for cfg in ${CONFIGS:-c3}; do
      BWRT_LIB=$L timeout -k 10 180 python bench.py --no-cpu-baseline --config $cfg --steps ${STEPS:-20} --warmup 3 \
          > $OUT/b_${label}_$cfg.log 2>&1 || { echo "$label $cfg failed"; tail -3 $OUT/b_${label}_$cfg.log; exit 1; }
      echo "$label $cfg $(grep -o '"kernel_ms_avg[^,]*' $OUT/b_${label}_$cfg.log)"
    done
    [ -n "${STRIDES-1,4,8,16}" ] && { BWRT_LIB=$L timeout -k 10 180 python tools/shard_sweep.py --config c3 --strides ${STRIDES:-1,4,8,16} \
        --blocks 0 --reps 10 2>&1 | grep stride | sed "s/^/$label /" || exit 1; }
  done
done
