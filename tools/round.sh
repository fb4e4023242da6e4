#!/bin/bash
# One GPU-box check of HEAD (run from the repo root): GPU suite, smoke, bench
# with the CPU baseline, c3 / c2 row-shard sweeps, and the plain-launch N = 2
# rehearsal (python bench.py --gpus 2: bench.py starts its own two ranks,
# here sharing the one GPU over gloo).  Every GPU step has its own time limit
# and the chain stops at the first failure.
# usage: tools/round.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-r05}; OUT=gpurun_out/$TAG; mkdir -p $OUT
K=(); [ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest_gpu rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc = 0 ] || { tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
for c in c3:1,2,4,6,8,16 c2:1,2,4,8; do
  BWRT_TUNING=1 timeout -k 10 200 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 > $OUT/shards_${c%:*}.txt 2>&1 || { echo "shards ${c%:*} failed"; exit 1; }
  grep stride $OUT/shards_${c%:*}.txt
done
BWRT_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > $OUT/self_launch_2.log 2>&1 || { echo "self-launch failed"; tail -20 $OUT/self_launch_2.log; exit 1; }
grep -o '"world_size[^,]*\|"verified[^,]*\|"ms_per_step[^,]*' $OUT/self_launch_2.log | tr '\n' ' '; echo
