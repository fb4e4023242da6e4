#!/bin/bash
# Wave-tile shapes for the pair kernel's small shards (BWRT_TILE = tile width:
# 32 x 2 is the launch policy's small-shard tile, 8 x 8 and 16 x 4 the others)
export BWRT_TUNING=1
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/shard_sweep.py --config c3 --strides 8,16 --blocks 0 --tiles 32,16,8,64 --reps 20 2>&1 | grep stride || exit 1
done
