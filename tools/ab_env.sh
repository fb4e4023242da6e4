#!/bin/bash
# A/B of (variant library, environment) pairs on the GPU box, alternating
# bench runs.  usage: ROUNDS=3 CONFIG=c3 bash tools/ab_env.sh "label:variant:ENV=1,ENV2=2" ...
# (variant "base" = lib/libbwrt.so; env list may be empty)
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
mkdir -p gpurun_out/ab_env
for r in $(seq ${ROUNDS:-3}); do
  for spec in "$@"; do
    IFS=: read -r label var envs <<< "$spec"
    L=$V/$var/libbwrt.so; [ "$var" = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
    env BWRT_LIB=$L ${envs//,/ } timeout -k 10 180 python bench.py --no-cpu-baseline --config ${CONFIG:-c3} \
        --steps ${STEPS:-20} --warmup 3 > gpurun_out/ab_env/b_$label.log 2>&1 || { echo "$label failed"; tail -3 gpurun_out/ab_env/b_$label.log; exit 1; }
    echo "$label $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/ab_env/b_$label.log)"
  done
done
