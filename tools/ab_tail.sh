#!/bin/bash
# Tail-mode A/B on c3: parity subset with the working library, then alternating
# full-frame benches and row-shard sweeps: HEAD variant vs the working library at
# several BWRT_TAIL thresholds (NAME@T: variant NAME).  usage: [TAILS="0 4 16 tailnc@4"] [ROUNDS=2] bash tools/ab_tail.sh
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
OUT=gpurun_out/ab_tail; mkdir -p $OUT
V=$PWD/bwidman-raytracer_amd/build/variants
timeout -k 10 500 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread \
    -k "${SUBSET:-tail or config3 or config2 or 07_small or quads or random or ragged or bounce or shards or repeated or global_records}" \
    > $OUT/pt.log 2>&1; rc=$?; echo "parity: $(tail -1 $OUT/pt.log)"; [ $rc = 0 ] || { tail -30 $OUT/pt.log; exit 1; }
for r in $(seq ${ROUNDS:-2}); do
  for v in ${TAILS:-0 4 16}; do
    # token T = the working library at BWRT_TAIL=T; NAME@T = build/variants/NAME at T
    case $v in *@*) L=$V/${v%@*}/libbwrt.so; T=${v#*@};; *) L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so; T=$v;; esac
    BWRT_TAIL=$T BWRT_LIB=$L timeout -k 10 120 python bench.py --no-cpu-baseline > $OUT/b_$v.log 2>&1 || { tail -5 $OUT/b_$v.log; exit 1; }
    echo "$v $(grep -o '"kernel_ms_avg[^,]*' $OUT/b_$v.log)"
    BWRT_TAIL=$T BWRT_LIB=$L timeout -k 10 120 python tools/shard_sweep.py --config c3 --strides ${STRIDES:-4,8,16} --blocks 0 --reps 10 2>&1 | grep stride | sed "s/^/$v /" || exit 1
  done
done
