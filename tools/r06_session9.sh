#!/bin/bash
# Round-6 GPU session 9: what the cold-start transient is — config 3, 200
# launches, re-seeding the RNG before launch 100 (an RNG transient comes
# back) or idling the GPU 200 ms before it (a clock transient comes back).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06i; mkdir -p $O
timeout -k 10 200 python tools/clock_ramp.py 200 --reseed-at 100 > $O/ramp_reseed.txt 2>&1 || exit 1
timeout -k 10 200 python tools/clock_ramp.py 200 --pause-at 100 > $O/ramp_pause.txt 2>&1 || exit 1
echo done > $O/done.txt
