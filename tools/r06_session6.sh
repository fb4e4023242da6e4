#!/bin/bash
# Round-6 GPU session 6: HEAD check after the stream-priority change — the
# whole GPU suite, smoke(), the bench (c3 with CPU baseline and oracle
# check, c5), the --dist path at world 1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 > $O/bench_c5.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --dist --steps 20 --warmup 5 > $O/bench_dist1.log 2>&1 || exit 1
timeout -k 10 300 python tools/shard_sweep.py --config c3 --strides 1,2,4,8 --blocks 0 --reps 20 > $O/shards_c3.txt 2>&1 || exit 1
echo done > $O/done.txt
