#!/bin/bash
# Round-6 GPU session 3: config-3 A/B of I-phase issue priority (ip2_48 /
# ip2_32: s_setprio 2 for waves with >= 48 / 32 rays during the closest hit)
# and an -O2 build of the brute-force kernels, full frame and shards.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06c; mkdir -p $O
SUBSET="config3_07_full or config3_shards" timeout -k 10 400 bash tools/ab.sh "o2:o2:" > $O/parity_o2.txt 2>&1 || exit 1
ROUNDS=3 MODE=bench timeout -k 10 400 bash tools/ab.sh "head:base:" "ip48:ip2_48:" "ip32:ip2_32:" "o2:o2:" > $O/ab_c3.txt 2>&1 || exit 1
ROUNDS=2 MODE=shard STRIDES=2,4,8 timeout -k 10 400 bash tools/ab.sh "head:base:" "ip48:ip2_48:" "ip32:ip2_32:" "o2:o2:" > $O/ab_shards.txt 2>&1 || exit 1
echo done > $O/done.txt
