#!/bin/bash
# c5 (BVH refill kernel) A/B on the GPU box: the BVH / stress parity subset
# with each candidate library, then alternating c5 bench runs over leaf-batch
# thresholds.  usage: LIBS="base park1" BATCHES="60 48" ROUNDS=2 bash tools/ab_c5.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
mkdir -p gpurun_out/ab_c5
lib_of() { [ "$1" = base ] && echo $PWD/bwidman-raytracer_amd/lib/libbwrt.so || echo $V/$1/libbwrt.so; }
for v in ${LIBS:-base}; do
  [ "$v" = base ] && continue
  BWRT_LIB=$(lib_of $v) timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
      -k "${SUBSET:-stress or bvh or random or config5}" > gpurun_out/ab_c5/pt_$v.log 2>&1; rc=$?
  echo "$v parity: $(tail -1 gpurun_out/ab_c5/pt_$v.log)"; [ $rc = 0 ] || exit 1
done
for r in $(seq ${ROUNDS:-2}); do
  for b in ${BATCHES:-60}; do
    for v in ${LIBS:-base}; do
      BWRT_LEAF_BATCH=$b BWRT_LIB=$(lib_of $v) timeout -k 10 120 python bench.py --no-cpu-baseline --config c5 \
          --steps ${STEPS:-3} --warmup 1 ${EXTRA:-} > gpurun_out/ab_c5/b_${v}_$b.log 2>&1 || { echo "bench $v $b failed"; tail -3 gpurun_out/ab_c5/b_${v}_$b.log; exit 1; }
      echo "$v batch=$b $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/ab_c5/b_${v}_$b.log)"
    done
  done
done
