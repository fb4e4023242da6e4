#!/bin/bash
# Round-6 GPU session 11: steady-state A/B (40 warm-up steps) of config-3
# micro-levers: SPEC-wave issue priority 0 / 1 (product 3), 6 waves per SIMD
# for the global-record kernel (product 7), one LDS record level (product 2),
# and the runtime knobs order period 4 / 64 (product 16), wave tiles 16x4 /
# 4x16 (product 8x8), launch-order feedback off; the brute-force loop
# unrolled 2 / 3 / 6 times (RT_HIT_UNROLL).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06k; mkdir -p $O
WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 900 bash tools/ab.sh "head:base:" "sp0:sp0:" "sp1:sp1:" \
    "gw6:gw6:" "ll1:ll1:" "u2:u2:" "u3:u3:" "u6:u6:" > $O/ab_steady_build.txt 2>&1 || exit 1
WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 900 bash tools/ab.sh "head:base:" "op4:base:BWRT_ORDER_PERIOD=4" \
    "op64:base:BWRT_ORDER_PERIOD=64" "t16:base:BWRT_TILE=16" "t4:base:BWRT_TILE=4" "noord:base:BWRT_ORDER=0" \
    > $O/ab_steady_knobs.txt 2>&1 || exit 1
echo done > $O/done.txt
