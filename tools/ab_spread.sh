#!/bin/bash
# Spread-launch A/B on c3 (BWRT_SPREAD=1: block/2 pixels per group, RANDDIR and
# SPEC tasks in different waves): parity subset, then alternating row-shard
# sweeps: the launch policy vs spread 256/128 vs spread 128/64.
# usage: [ROUNDS=2] [STRIDES=1,2,4,8,16] bash tools/ab_spread.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
OUT=gpurun_out/ab_spread; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread \
    -k "${SUBSET:-spread or tail or config3 or 07_small or quads or shards or launch_order_feedback}" \
    > $OUT/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { tail -30 $OUT/pt.log; exit 1; }
for r in $(seq ${ROUNDS:-2}); do
  for v in policy:0:0 s256:1:256 s128:1:128; do
    IFS=: read name sp blk <<< "$v"
    BWRT_SPREAD=$sp timeout -k 10 150 python tools/shard_sweep.py --config c3 --strides ${STRIDES:-1,2,4,8,16} --blocks $blk --reps 10 2>&1 | grep stride | sed "s/^/$name /" || exit 1
  done
done
