#!/bin/bash
# Round-6 GPU session 12: three LDS record levels for the global-record
# kernel (build/variants/ll3; product 2) in steady state, configs 3 and 4.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06l; mkdir -p $O
WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "ll3:ll3:" > $O/ab_steady_ll3_c3.txt 2>&1 || exit 1
CONFIG=c4 WARMUP=10 STEPS=10 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "ll3:ll3:" > $O/ab_steady_ll3_c4.txt 2>&1 || exit 1
echo done > $O/done.txt
