#!/bin/bash
# Pair-kernel wave priority for the costliest groups (launch-order feedback on
# a resident grid): the working library vs build/variants/{noprio,prio3,div2}.
# usage: [ROUNDS=2] bash tools/ab_prio.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
OUT=gpurun_out/ab_prio; mkdir -p $OUT
V=$PWD/bwidman-raytracer_amd/build/variants
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread \
    -k "${SUBSET:-spread or shards or 07_small or config1 or launch_order}" \
    > $OUT/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { tail -30 $OUT/pt.log; exit 1; }
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARS:-main noprio prio3 div2}; do
    if [ $v = main ]; then L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so; else L=$V/$v/libbwrt.so; fi
    for c in c3:8,16 c2:8; do
      BWRT_LIB=$L timeout -k 10 150 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 30 2>&1 | grep stride | sed "s/^/$v /" || exit 1
    done
  done
done
