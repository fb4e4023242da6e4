#!/bin/bash
# Round-6 GPU session 5: the multi-rank step at world size 1 (one process,
# env:// rendezvous): serial vs pipelined gather, the render stream at high
# priority (BWRT_STREAM_PRIO=1), the de-interleave grid capped
# (BWRT_DEINT_BLOCKS); two alternating rounds, 50 steps each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread \
    -k "deinterleave or render_device_into_torch" > $O/pt_deint.log 2>&1 || exit 1
export BWRT_TUNING=1
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 5 "$@" > $O/$label.log 2>&1 \
      || { echo "$label failed"; tail -3 $O/$label.log; return 1; }
  echo "$label $(grep -o '"ms_per_step[^,]*' $O/$label.log) $(grep -o '"kernel_ms_avg[^,]*' $O/$label.log) $(grep -o '"verified[^,]*' $O/$label.log)" | tee -a $O/summary.txt
}
D=(WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517)
for r in 1 2; do
  run plain_$r BWRT_X=0 -- || exit 1
  run plain_prio_$r BWRT_STREAM_PRIO=1 -- || exit 1
  run serial_$r "${D[@]}" -- --gpus 1 --dist --no-overlap || exit 1
  run serial_prio_$r "${D[@]}" BWRT_STREAM_PRIO=1 -- --gpus 1 --dist --no-overlap || exit 1
  run overlap_$r "${D[@]}" -- --gpus 1 --dist || exit 1
  run overlap_prio_$r "${D[@]}" BWRT_STREAM_PRIO=1 -- --gpus 1 --dist || exit 1
  run overlap_prio_d256_$r "${D[@]}" BWRT_STREAM_PRIO=1 BWRT_DEINT_BLOCKS=256 -- --gpus 1 --dist || exit 1
  run overlap_d64_$r "${D[@]}" BWRT_DEINT_BLOCKS=64 -- --gpus 1 --dist || exit 1
done
echo done > $O/done.txt
