#!/bin/bash
# PMC passes for the bench workload (run on the GPU box from the repo root).
# Usage: tools/pmc.sh OUTDIR [bench args...]
# Counters are collected in SEPARATE passes (FETCH_SIZE and WRITE_SIZE cannot
# share one; MI355X_MICROARCH.md §rocprofv3 PMC slots), kernel-trace only.
set -o pipefail
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d "$OUT/pass$i" -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline "$@" > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($set) failed"; tail -5 "$OUT/pass$i.log"; }
done
