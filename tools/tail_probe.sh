#!/bin/bash
# Tail-mode diagnostics: RT_STAMPS phase / tail counters (stamps variant:
# tools/variants.sh stamps -DRT_STAMPS) at row strides 8 / 64 with the tail
# off and on.  stamps[0..7] main-loop phase cycles, [8] rounds, [32] tail
# cycles, [33] tail rounds, [34] tail entries, [35] pixels handed over.
export BWRT_TUNING=1
mkdir -p gpurun_out/tail_probe
for t in ${TAILS:-0 4 16}; do
  for g in ${STRIDES:-8 64}; do
    BWRT_TAIL=$t BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/stamps/libbwrt.so timeout -k 10 120 \
        python tools/stamps_run.py $g > gpurun_out/tail_probe/st_t${t}_g$g.log 2>&1 || { tail -5 gpurun_out/tail_probe/st_t${t}_g$g.log; exit 1; }
    echo "tail=$t stride=$g $(grep stamps gpurun_out/tail_probe/st_t${t}_g$g.log)"
  done
done
