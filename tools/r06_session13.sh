#!/bin/bash
# Round-6 GPU session 13: config-3 shards (1/4, 1/8) under other wave tiles,
# 100 launches per point in one process (the policy's tiles first, cold, and
# again last, warm).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 600 python tools/shard_sweep.py --config c3 --strides 4,8 --blocks 0 --tiles=-1,64,32,16,8,4,-1 --reps 100 \
    > $O/shards_tiles.txt 2>&1 || exit 1
echo done > $O/done.txt
