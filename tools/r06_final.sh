#!/bin/bash
# Round-6 final HEAD check: the whole GPU suite, smoke(), the default bench
# (the driver's command), and the --dist path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=${OUT:-gpurun_out/r06z}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --dist --steps 20 --warmup 5 > $O/bench_dist1.log 2>&1 || exit 1
echo done > $O/done.txt
