#!/bin/bash
# Round-6 GPU session 10: steady-state A/B (40 warm-up steps, past the
# cold-start ramp) of the config-3 candidates measured flat in the ramp:
# I-phase issue priority (ip2_48, ip2_32) and -O2 (o2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06j; mkdir -p $O
WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "ip48:ip2_48:" "ip32:ip2_32:" "o2:o2:" > $O/ab_steady_c3.txt 2>&1 || exit 1
echo done > $O/done.txt
# the 8-wave global-record shape at full frame in steady state (build/variants/g8:
# profiles/r06a/grec8_shape.diff re-applied), against the 7-wave one, same library
WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "g7:g8:BWRT_GREC=1" "g8:g8:BWRT_GREC=2" > $O/ab_steady_g8.txt 2>&1 || exit 1
echo done2 > $O/done2.txt
