#!/bin/bash
# A/B timing on the GPU box: tools/ab.sh "ENV=.. ENV2=..|label" ...  (bench.py, no CPU baseline)
for cfg in "$@"; do
  envs=${cfg%%|*}; label=${cfg##*|}
  env $envs timeout -k 10 120 python bench.py --no-cpu-baseline "${AB_ARGS[@]}" > gpurun_out/ab.log 2>&1
  echo "$label $(tail -1 gpurun_out/ab.log | grep -o '"ms_per_step[^,]*')"
done
