#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench (with CPU baseline), rocprof
# kernel-trace stats and PMC passes for the bench workload.  Every GPU step
# has its own time limit and the chain stops at the first failure.
# usage (on the box, from the repo root): tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest_gpu rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo rocprof failed; tail -5 $OUT/prof.log; exit 1; }
tools/pmc.sh $OUT/pmc --steps 5 --warmup 1
echo done
