#!/bin/bash
# Split closest hit (spread groups: the executor wave takes half of every
# closest hit) vs the same build without it (build/variants/nosplit):
# parity, then alternating c3 / c2 small-shard sweeps.  usage: [ROUNDS=2] bash tools/ab_split.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
OUT=gpurun_out/ab_split; mkdir -p $OUT
V=$PWD/bwidman-raytracer_amd/build/variants
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread \
    -k "${SUBSET:-spread or shards or 07_small or quads or config1 or random or scaled or ragged or tail}" \
    > $OUT/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { tail -30 $OUT/pt.log; exit 1; }
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARS:-split nosplit}; do
    if [ $v = split ] || [ $v = main ]; then L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so; else L=$V/$v/libbwrt.so; fi
    for c in c3:8,16 c2:8,16; do
      BWRT_LIB=$L timeout -k 10 150 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 2>&1 | grep stride | sed "s/^/$v /" || exit 1
    done
  done
done
