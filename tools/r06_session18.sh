#!/bin/bash
# Round-6 GPU session 18: a global record's fold read non-temporal
# (RT_NT_GREC=1) against HEAD: parity subset, steady-state configs 3 and 4.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06u; mkdir -p $O
SUBSET="config3 or config4 or global_records or deep" WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench \
    timeout -k 10 900 bash tools/ab.sh "head:base:" "ng:ng:" > $O/ab_steady_ng_c3.txt 2>&1 || exit 1
CONFIG=c4 WARMUP=10 STEPS=10 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "ng:ng:" \
    > $O/ab_steady_ng_c4.txt 2>&1 || exit 1
cp gpurun_out/ab/pt_*.log $O/
echo done > $O/done.txt
