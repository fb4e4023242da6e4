#!/bin/bash
# PMC A/B of the render kernel (GPU box, repo root): one counter pass per
# candidate ("label:variant:ENV=1,ENV2=2" as tools/ab.sh), the bench workload
# ($CONFIG, default c3), then tools/pmc_summary.py per candidate.
# COUNTERS overrides the default set (at most 8 SQ_ counters in one pass).
export BWRT_TUNING=1
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_ab}; mkdir -p $OUT
V=$PWD/bwidman-raytracer_amd/build/variants
CNT=${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for spec in "$@"; do
  IFS=: read -r label var envs <<< "$spec"
  L=$V/$var/libbwrt.so; [ "$var" = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
  rm -rf $OUT/$label; mkdir -p $OUT/$label
  env BWRT_LIB=$L ${envs//,/ } timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT -d $OUT/$label/pass1 -o run \
      --output-format csv -- python3 bench.py --no-cpu-baseline --config ${CONFIG:-c3} --steps 5 --warmup 1 \
      > $OUT/$label.log 2>&1 || { echo "$label failed"; tail -5 $OUT/$label.log; exit 1; }
  echo "== $label"; python3 tools/pmc_summary.py $OUT/$label ${KERNEL:-rt_render} | tr -d '\n' | sed 's/  */ /g'; echo
done
