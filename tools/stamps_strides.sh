#!/bin/bash
# RT_STAMPS phase counters of the sorted kernel at row strides 1 / 8 / 64 (build the
# stamps variant first: tools/variants.sh stamps -DRT_STAMPS), then the shard sweep
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
for g in 1 8 64; do
  BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/stamps/libbwrt.so timeout -k 10 120 python tools/stamps_run.py $g > gpurun_out/st$g.log 2>&1 || { tail -5 gpurun_out/st$g.log; exit 1; }
  echo "stride=$g"; grep stamps gpurun_out/st$g.log
done
python tools/shard_sweep.py --strides 1,8,64 --blocks 0 --reps 10
