#!/bin/bash
# c3 A/B of a variant library (tools/variants.sh NAME): the config-3 parity
# subset, then alternating full-frame benches and shard sweeps.
# usage: CAND=name [ROUNDS=3] [STRIDES=1,4,8] bash tools/ab_c3.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
mkdir -p gpurun_out/ab_c3
BWRT_LIB=$V/$CAND/libbwrt.so timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -k "${SUBSET:-config3 or config1 or config2 or 07_small or quads or random or ragged or bounce or shards or repeated}" \
    > gpurun_out/ab_c3/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 gpurun_out/ab_c3/pt.log)"; [ $rc = 0 ] || exit 1
for r in $(seq ${ROUNDS:-3}); do
  for v in base $CAND; do
    L=$V/$v/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
    BWRT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/ab_c3/b_$v.log 2>&1 || exit 1
    echo "$v $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/ab_c3/b_$v.log)"
    BWRT_LIB=$L timeout -k 10 120 python tools/shard_sweep.py --config c3 --strides ${STRIDES:-4,8} --blocks 0 --reps 10 2>&1 | grep stride | sed "s/^/$v /"
  done
done
