#!/bin/bash
# One PMC pass per variant on c3 row shards: the pair kernel (policy) vs the
# sorted spread kernel (BWRT_PAIR=0): instructions, lane-cycles, waits.
# usage (GPU box, repo root): tools/pmc_pair.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/pmc_pair}
export BWRT_TUNING=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for g in 8 16; do
  for p in 1 0; do
    BWRT_PAIR=$p timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        -d "$OUT/g${g}_p$p" -o run --output-format csv -- \
        python3 tools/shard_sweep.py --config c3 --blocks 0 --strides $g --reps 5 > "$OUT/g${g}_p$p.log" 2>&1 || { echo "pmc g=$g pair=$p failed"; tail -5 "$OUT/g${g}_p$p.log"; exit 1; }
    echo "g=$g pair=$p done"
  done
done
