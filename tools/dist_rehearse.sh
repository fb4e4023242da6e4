#!/bin/bash
# Rehearse bench.py's N > 1 path on one GPU box: 2 and 3 ranks sharing the GPU over
# gloo (staged through the host), with and without frame pipelining, --verify
# checks the gathered frame against a 1-GPU render.  Then a shard sweep and the N=1 bench.
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
mkdir -p gpurun_out
for n in 2 3; do
  for ov in "" "--no-overlap"; do
    BWRT_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $n --steps 10 --warmup 3 $ov > gpurun_out/dist_$n$ov.log 2>&1 || { echo "FAIL $n $ov"; tail -20 gpurun_out/dist_$n$ov.log; exit 1; }
    echo "n=$n $ov: $(grep -o '"ms_per_step[^,]*' gpurun_out/dist_$n$ov.log) $(grep -o '"verified[^,]*' gpurun_out/dist_$n$ov.log) $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/dist_$n$ov.log)"
    grep -q '"verified": true' gpurun_out/dist_$n$ov.log || { echo "not verified"; exit 1; }
  done
done
timeout -k 10 100 python -u tools/shard_sweep.py --blocks 0 --strides 1,2,4,8 2>&1 | grep -v amdgpu.ids
timeout -k 10 100 python bench.py --no-cpu-baseline 2>&1 | tail -1
