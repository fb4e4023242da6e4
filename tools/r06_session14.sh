#!/bin/bash
# Round-6 GPU session 14: non-temporal pixel-state streams (RT_NT_PIXEL=1)
# against HEAD — parity subset, then steady-state A/B on config 3 and 4, and
# the shards.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06q; mkdir -p $O
SUBSET="config3 or shard or spread or deinterleave or stress" WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench \
    timeout -k 10 900 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_steady_nt_c3.txt 2>&1 || exit 1
CONFIG=c4 WARMUP=10 STEPS=10 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" \
    > $O/ab_steady_nt_c4.txt 2>&1 || exit 1
cp gpurun_out/ab/pt_*.log $O/ 2>/dev/null
echo done > $O/done.txt
