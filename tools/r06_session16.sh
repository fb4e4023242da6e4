#!/bin/bash
# Round-6 GPU session 16: non-temporal pixel loads / stores / both
# (RT_NT_PIXEL = 1 / 2 / 3) against HEAD, steady state; then HEAD vs both in
# the driver's window (5 + 20 steps)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06s; mkdir -p $O
WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 900 bash tools/ab.sh "head:base:" "ntl:ntl:" "nts:nts:" "nt:nt:" \
    > $O/ab_steady_nt3_c3.txt 2>&1 || exit 1
WARMUP=5 STEPS=20 ROUNDS=4 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_window_nt_c3.txt 2>&1 || exit 1
echo done > $O/done.txt
