#!/bin/bash
# Per-step overhead A/B: bench renders on the context's own stream (deferred
# end event, the default) vs on a torch-created stream (an end event recorded
# after every launch: BENCH_CALLER_STREAM=1), alternating, configs c2 and c3.
set -o pipefail
for r in 1 2 3; do
  for cfg in c2 c3; do
    for cs in 0 1; do
      BENCH_CALLER_STREAM=$cs timeout -k 10 120 python bench.py --config $cfg --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/ab_stream.log 2>&1 || { tail -3 gpurun_out/ab_stream.log; exit 1; }
      echo "$cfg caller_stream=$cs $(grep -o '"ms_per_step[^,]*' gpurun_out/ab_stream.log) $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/ab_stream.log)"
    done
  done
done
