#!/bin/bash
# Pair kernel (spread launches: owner wave + helper wave, 3 barriers a round)
# vs spread launches through the sorted kernel (BWRT_PAIR=0): parity, then
# alternating small-shard sweeps.  usage: [ROUNDS=2] bash tools/ab_pair.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
OUT=gpurun_out/ab_pair; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread \
    -k "${SUBSET:-spread or shards or 07_small or quads or config1 or random or scaled or ragged or bounce or repeated or samples}" \
    > $OUT/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { tail -30 $OUT/pt.log; exit 1; }
for r in $(seq ${ROUNDS:-2}); do
  for p in 1 0; do
    for c in c3:6,8,16 c2:4,8,16; do
      BWRT_PAIR=$p timeout -k 10 150 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 2>&1 | grep stride | sed "s/^/pair=$p /" || exit 1
    done
  done
done
