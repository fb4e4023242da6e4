#!/bin/bash
# Round-6 GPU session 19: the final HEAD set after the non-temporal pixel
# streams — config-3 and config-5 PMC passes (traffic records), rocprof
# kernel stats of the c3 bench, the whole GPU suite, smoke(), the benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06v; mkdir -p $O
step() { echo "== $(date +%T) $1" >> $O/steps.txt; }
step pmc-c3
timeout -k 10 500 bash tools/pmc.sh $O/pmc_c3 --config c3 --steps 3 --warmup 1 > $O/pmc_c3.log 2>&1 || exit 1
python3 tools/make_traffic_json.py $O/pmc_c3 07-1920x1080-8spp-4b-rows1 $O/traffic_c3.json > /dev/null || exit 1
step pmc-c5
timeout -k 10 500 bash tools/pmc.sh $O/pmc_c5 --config c5 --steps 1 --warmup 1 > $O/pmc_c5.log 2>&1 || exit 1
python3 tools/make_traffic_json.py $O/pmc_c5 stress-1920x1080-32spp-8b-rows1 $O/traffic_c5.json > /dev/null || exit 1
step pytest-gpu
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
step smoke
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
step bench-c3
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --traffic-json $O/traffic_c3.json > $O/bench.log 2>&1 || exit 1
step rocprof-c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c3 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --traffic-json $O/traffic_c3.json > $O/rocprof_c3_bench.log 2>&1 || exit 1
step bench-c5
timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 --traffic-json $O/traffic_c5.json > $O/bench_c5.log 2>&1 || exit 1
step bench-dist
timeout -k 10 300 python3 bench.py --gpus 1 --dist --steps 20 --warmup 5 > $O/bench_dist1.log 2>&1 || exit 1
step done
