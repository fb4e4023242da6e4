#!/bin/bash
# Round-6 GPU session 2 (run on the GPU box from the repo root): c5 A/B of
# this tree against the round-5 HEAD library (build/variants/r5: the 16-byte
# nodes' alignment and the diagnostics move), config-5 PMC passes for its
# traffic record (HBM + L1 lines), the whole GPU suite, the bench for c3 and
# c5, and rocprof kernel stats of the c3 bench.  First failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06b; mkdir -p $O
step() { echo "== $(date +%T) $1" >> $O/steps.txt; }
step ab-c5-r5
ROUNDS=3 MODE=bench CONFIG=c5 STEPS=5 timeout -k 10 400 bash tools/ab.sh "head:base:" "r5:r5:" > $O/ab_c5_r5.txt 2>&1 || exit 1
step pmc-c5
timeout -k 10 500 bash tools/pmc.sh $O/pmc_c5 --config c5 --steps 1 --warmup 1 > $O/pmc_c5.log 2>&1 || exit 1
python3 tools/make_traffic_json.py $O/pmc_c5 stress-1920x1080-32spp-8b-rows1 $O/traffic_c5.json > /dev/null || exit 1
step pytest-gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
step bench-c3
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 1
step bench-c5
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --traffic-json $O/traffic_c5.json > $O/bench_c5.log 2>&1 || exit 1
step rocprof-c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline > $O/rocprof_bench.log 2>&1 || exit 1
step done
