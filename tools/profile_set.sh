#!/bin/bash
# The round's profile set of the bench workload (GPU box, repo root), after
# tools/round.sh TAG: rocprofv3 kernel-trace stats of the bench, the PMC
# passes (tools/pmc.sh) and, when the RT_PHASE_TWICE variants are built
# (tools/variants.sh ph1 -DRT_PHASE_TWICE=1 ... ph4), the per-phase lanes.
set -o pipefail
TAG=${1:-r05}; OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo rocprof failed; tail -5 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log | cut -c1-200
bash tools/pmc.sh $OUT/pmc --steps 5 --warmup 1 || exit 1
python3 tools/pmc_summary.py $OUT/pmc rt_render_sorted | tr -d '\n' | cut -c1-600; echo
if [ -f bwidman-raytracer_amd/build/variants/ph4/libbwrt.so ]; then
  bash tools/phase_lanes.sh $OUT/phase_lanes > $OUT/phase_lanes.txt 2>&1 || { echo phase lanes failed; tail -5 $OUT/phase_lanes.txt; exit 1; }
  tail -40 $OUT/phase_lanes.txt
fi
