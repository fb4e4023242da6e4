#!/bin/bash
# Deferred-fold A/B: GPU parity of the working library (full suite), then
# alternating benches of configs 3 and 4 (global-record launches: the deferred
# fold applies) against the RT_DEFER_FOLD=0 variant (tools/variants.sh nodf -DRT_DEFER_FOLD=0)
export BWRT_TUNING=1
set -o pipefail
OUT=gpurun_out/ab_df; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pt.log 2>&1; rc=$?
echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { grep -E "FAILED|Error" $OUT/pt.log | head; exit 1; }
V=$PWD/bwidman-raytracer_amd/build/variants
for r in 1 2 3; do
  for v in nodf df; do
    L=$V/nodf/libbwrt.so; [ $v = df ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
    for cfg in c3 c4; do
      BWRT_LIB=$L timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 30 --warmup 5 > $OUT/b.log 2>&1 || { tail -3 $OUT/b.log; exit 1; }
      echo "$v $cfg $(grep -o '"ms_per_step[^,]*' $OUT/b.log) $(grep -o '"kernel_ms_avg[^,]*' $OUT/b.log)"
    done
  done
done
