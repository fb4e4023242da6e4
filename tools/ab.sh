#!/bin/bash
# A/B timing on the GPU box (run from the repo root), alternating candidates
# over ROUNDS rounds.  A candidate is "label:variant:ENV=1,ENV2=2":
#   variant  a library built by tools/variants.sh (build/variants/<name>),
#            or "base" = the working bwidman-raytracer_amd/lib/libbwrt.so;
#   ENV list launch knobs for that run (may be empty; BWRT_TUNING=1 is set).
# MODE=bench  (default) bench.py --config $CONFIG (c3): kernel_ms_avg, ms/step
# MODE=shard  tools/shard_sweep.py --config $CONFIG --strides $STRIDES
# SUBSET=expr first runs `pytest -m gpu -k expr` with every candidate library
#             (the parity gate of an A/B; SUBSET=all: the whole GPU suite).
# WARMUP=k    bench warm-up steps (default 3): a GPU idle between runs comes
#             back through a ~20-launch power-management ramp (DESIGN.md §5,
#             "Cold-start transient"); WARMUP=40 compares steady states
# usage: ROUNDS=3 MODE=bench CONFIG=c3 bash tools/ab.sh "head:base:" "cand:myvar:"
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
OUT=gpurun_out/ab; mkdir -p $OUT
lib_of() { [ "$1" = base ] && echo $PWD/bwidman-raytracer_amd/lib/libbwrt.so || echo $V/$1/libbwrt.so; }
if [ -n "$SUBSET" ]; then
  for spec in "$@"; do
    IFS=: read -r label var envs <<< "$spec"
    K=(); [ "$SUBSET" = all ] || K=(-k "$SUBSET")
    # the knobs go through BWRT_AB_ENV: tests/conftest.py strips every other
    # BWRT_* variable before the tests run
    env BWRT_LIB=$(lib_of $var) BWRT_AB_ENV="$envs" timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 \
        --timeout-method thread "${K[@]}" > $OUT/pt_$label.log 2>&1 || { echo "$label parity FAILED"; tail -5 $OUT/pt_$label.log; exit 1; }
    echo "$label parity: $(tail -1 $OUT/pt_$label.log)"
  done
fi
for r in $(seq ${ROUNDS:-3}); do
  for spec in "$@"; do
    IFS=: read -r label var envs <<< "$spec"
    if [ "${MODE:-bench}" = shard ]; then
      env BWRT_LIB=$(lib_of $var) ${envs//,/ } timeout -k 10 200 python tools/shard_sweep.py --config ${CONFIG:-c3} \
          --strides ${STRIDES:-4,8} --blocks 0 --reps ${REPS:-20} > $OUT/s_$label.log 2>&1 || { echo "$label failed"; tail -3 $OUT/s_$label.log; exit 1; }
      grep stride $OUT/s_$label.log | sed "s/^/$label /"
    else
      env BWRT_LIB=$(lib_of $var) ${envs//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline --config ${CONFIG:-c3} \
          --steps ${STEPS:-20} --warmup ${WARMUP:-3} > $OUT/b_$label.log 2>&1 || { echo "$label failed"; tail -3 $OUT/b_$label.log; exit 1; }
      echo "$label $(grep -o '"kernel_ms_avg[^,]*' $OUT/b_$label.log) $(grep -o '"ms_per_step[^,]*' $OUT/b_$label.log)"
    fi
  done
done
