#!/bin/bash
# Memory-pipeline PMC passes (SQ / TA / TCP / TCC / TD) for one bench config, run on the GPU box
# from the repo root: tools/pmc_mem.sh [c5|c3]  -> gpurun_out/pmc5_<cfg>/pass*/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
CFG=${1:-c5}
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum TD_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d gpurun_out/pmc5_$CFG/pass$i -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --config $CFG --steps 1 --warmup 1 > gpurun_out/pmc5_$CFG.pass$i.log 2>&1 || { echo "pass $i failed"; tail -3 gpurun_out/pmc5_$CFG.pass$i.log; }
done
python3 tools/pmc_summary.py gpurun_out/pmc5_$CFG rt_render
