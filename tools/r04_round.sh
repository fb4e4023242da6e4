#!/bin/bash
# Round-4 profile set for the bench workload: GPU suite, smoke, bench with CPU
# baseline, rocprofv3 kernel-trace stats of the bench, PMC passes, the traffic /
# VALU summary bench.py reads, other configs' benches, row-shard sweeps.  Each GPU step has its
# own time limit; the chain stops at the first failure.
# usage (GPU box, repo root): tools/r04_round.sh TAG
set -o pipefail
TAG=${1:-r04b}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest_gpu rc=$rc: $(tail -1 $OUT/pytest_gpu.log)"; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log | grep smoke
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo bench failed; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo rocprof failed; tail -5 $OUT/prof.log; exit 1; }
tail -1 $OUT/prof.log | cut -c1-200
bash tools/pmc.sh $OUT/pmc --steps 5 --warmup 1 || exit 1
python3 tools/pmc_summary.py $OUT/pmc rt_render_sorted > $OUT/pmc_summary.json && \
python3 tools/make_traffic_json.py $OUT/pmc 07-1920x1080-8spp-4b-rows1 $OUT/traffic_latest.json || exit 1
for cfg in c2 c4 c5; do
  timeout -k 10 300 python bench.py --config $cfg > $OUT/bench_$cfg.log 2>&1 || { echo "bench $cfg failed"; tail -3 $OUT/bench_$cfg.log; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step[^,]*' $OUT/bench_$cfg.log)"
done
export BWRT_TUNING=1  # shard_sweep forces BWRT_BLOCK=0 (the launch policy)
for c in c3:1,2,4,8,16 c2:1,2,4,8,16 c4:2,4,8; do
  timeout -k 10 200 python tools/shard_sweep.py --config ${c%:*} --strides ${c#*:} --blocks 0 --reps 20 > $OUT/shards_${c%:*}.txt 2>&1 || { echo "shards ${c%:*} failed"; tail -3 $OUT/shards_${c%:*}.txt; exit 1; }
  grep stride $OUT/shards_${c%:*}.txt
done
echo done
