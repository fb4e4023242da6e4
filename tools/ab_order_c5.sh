#!/bin/bash
# c5 launch-order feedback A/B (refill kernel): parity subset, then alternating
# c5 benches with BWRT_ORDER=0 / 1.  usage: bash tools/ab_order_c5.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
mkdir -p gpurun_out/ord
timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -k "stress or bvh or random or config5 or order" > gpurun_out/ord/pt.log 2>&1; rc=$?
echo "parity: $(tail -1 gpurun_out/ord/pt.log)"; [ $rc = 0 ] || exit 1
for r in 1 2 3; do
  for o in 0 1; do
    BWRT_ORDER=$o timeout -k 10 120 python bench.py --no-cpu-baseline --config ${CFG:-c5} --steps ${STEPS:-5} --warmup 2 \
        > gpurun_out/ord/b_$o.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/ord/b_$o.log; exit 1; }
    echo "order=$o $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/ord/b_$o.log)"
  done
done
