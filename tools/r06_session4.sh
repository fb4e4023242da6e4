#!/bin/bash
# Round-6 GPU session 4: what the multi-rank step costs around the render at
# world size 1 (one process, env:// rendezvous, no launcher): the plain
# N = 1 bench, --dist with the pipelined gather, --dist --no-overlap, and a
# rocprof kernel trace of the --dist run (RCCL and de-interleave kernels).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/plain.log 2>&1 || exit 1
export WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
timeout -k 10 200 python bench.py --gpus 1 --dist --steps 50 --warmup 5 > $O/dist_overlap.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --gpus 1 --dist --no-overlap --steps 50 --warmup 5 > $O/dist_serial.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rp_dist -o run --output-format csv -- \
    python3 bench.py --gpus 1 --dist --steps 20 --warmup 5 > $O/rp_dist.log 2>&1 || exit 1
echo done > $O/done.txt
