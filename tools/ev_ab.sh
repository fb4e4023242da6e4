#!/bin/bash
# Cost of the marker packets between renders (bench.py config 3, 50 steps,
# alternating): library kernel timing on (start marker + end event per launch)
# vs off (end event only); the bench itself brackets its timed region with one
# event pair.  Then rocprofv3 kernel traces of both (gaps between launches).
# Round-3 results: profiles/r03d/launch_events/.
set -o pipefail
mkdir -p gpurun_out/ev
for r in 1 2 3; do
  for combo in "on:BENCH_KTIMING=1" "off:BENCH_KTIMING=0"; do
    IFS=: read -r label envs <<< "$combo"
    env $envs timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/ev/b_$label.log 2>&1 || { tail -3 gpurun_out/ev/b_$label.log; exit 1; }
    echo "$label $(grep -o '"ms_per_step[^,]*' gpurun_out/ev/b_$label.log) $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/ev/b_$label.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for label in on off; do
  v=0; [ $label = on ] && v=1
  BENCH_KTIMING=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ev/prof_$label -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/ev/prof_$label.log 2>&1 && echo "prof_$label ok" || exit 1
done
