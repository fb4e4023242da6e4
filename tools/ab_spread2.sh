#!/bin/bash
# Spread policy check: the full GPU suite, then row-shard sweeps of c2 / c3 / c4
# with the launch policy (spread on few-group launches) vs BWRT_SPREAD=0.
# usage: [ROUNDS=2] bash tools/ab_spread2.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
OUT=gpurun_out/ab_spread2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread \
    > $OUT/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { tail -30 $OUT/pt.log; exit 1; }
for r in $(seq ${ROUNDS:-2}); do
  for sp in policy 0; do
    for c in c2:1,2,4,8,16 c3:4,8,16 c4:8,16; do
      if [ $sp = policy ]; then unset BWRT_SPREAD; else export BWRT_SPREAD=$sp; fi
      timeout -k 10 150 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 10 2>&1 | grep stride | sed "s/^/spread=$sp /" || exit 1
    done
  done
done
unset BWRT_SPREAD
timeout -k 10 120 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log
