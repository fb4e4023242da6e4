#!/bin/bash
# Round-6 GPU session 8: the stream-priority test, and the per-launch render
# time against the shader clock from a cold start (tools/clock_ramp.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
    -k "stream_priority or deinterleave" > $O/pt.log 2>&1 || exit 1
timeout -k 10 200 python tools/clock_ramp.py 1500 > $O/clock_ramp_c3.txt 2>&1 || exit 1
timeout -k 10 200 python tools/clock_ramp.py 40 --config c5 > $O/clock_ramp_c5.txt 2>&1 || exit 1
echo done > $O/done.txt
