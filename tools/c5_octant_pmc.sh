#!/bin/bash
# Config 5 under different octant-array masks (BWRT_BVH_ORDER_MASK): kernel
# time and the memory counters that bound the walk (vector-memory read
# instructions, L1 tag accesses = lines per load, L1->L2 requests).
export BWRT_TUNING=1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/c5_octant; mkdir -p $OUT
for m in ${MASKS:-5 0 1 4 7}; do
  BWRT_BVH_ORDER_MASK=$m timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_WAVES TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE \
      -d $OUT/m$m -o run --output-format csv -- python3 bench.py --no-cpu-baseline --config c5 --steps 2 --warmup 1 > $OUT/m$m.log 2>&1 || { echo "mask $m failed"; tail -3 $OUT/m$m.log; exit 1; }
  echo "mask $m: $(grep -o '"kernel_ms_avg[^,]*' $OUT/m$m.log) $(python3 tools/pmc_summary.py $OUT/m$m rt_render | tr -d '\n ' )"
done
