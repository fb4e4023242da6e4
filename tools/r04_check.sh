#!/bin/bash
# round-4 check: full GPU suite, bench line, tail probe, per-phase lane breakdown
set -o pipefail
OUT=gpurun_out/r04a; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest_gpu rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc = 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
TAILS="0 4 16" bash tools/tail_probe.sh && SUBSET=tail_mode TAILS="0 4 8 16 tailnc@4 tailnc@16" ROUNDS=2 bash tools/ab_tail.sh && \
bash tools/phase_lanes.sh $OUT/phase_lanes && bash tools/ab_stream.sh && bash tools/dist_rehearse.sh
