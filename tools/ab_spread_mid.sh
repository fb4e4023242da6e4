#!/bin/bash
# Forced spread launches (the pair kernel since its addition) vs none at the
# mid-size shards, to place the launch policy's RT_SPREAD_PIX threshold.
export BWRT_TUNING=1
set -o pipefail
for r in 1 2; do for sp in 0 1; do
  for c in ${CFGS:-c3:2,3,4,6 c2:1,2,3}; do
    BWRT_SPREAD=$sp timeout -k 10 150 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 2>&1 | grep stride | sed "s/^/spread=$sp /" || exit 1
  done
done; done
