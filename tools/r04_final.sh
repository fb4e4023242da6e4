#!/bin/bash
# Final check of HEAD: GPU suite, smoke, bench, c3 / c2 shard sweeps.
# usage (GPU box, repo root): tools/r04_final.sh TAG
set -o pipefail
TAG=${1:-r04f}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest_gpu rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-250
export BWRT_TUNING=1
for c in c3:1,2,4,8,16 c2:1,2,4,8,16; do
  timeout -k 10 200 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 > $OUT/shards_${c%:*}.txt 2>&1 || { echo "shards ${c%:*} failed"; exit 1; }
  grep stride $OUT/shards_${c%:*}.txt
done
