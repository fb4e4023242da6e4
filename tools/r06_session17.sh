#!/bin/bash
# Round-6 GPU session 17: RT_NT_PIXEL=3 — the whole GPU suite on it, then the
# 1/4 and 1/8 shards of config 3 and config 4's 1/8 shard, three rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06t; mkdir -p $O
BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/nt/libbwrt.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread > $O/pytest_gpu_nt.log 2>&1 || exit 1
ROUNDS=3 MODE=shard STRIDES=4,8 timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_nt_shards_c3.txt 2>&1 || exit 1
CONFIG=c4 ROUNDS=2 MODE=shard STRIDES=8 timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_nt_shards_c4.txt 2>&1 || exit 1
echo done > $O/done.txt
