#!/bin/bash
# PMC passes for one row shard (stride G) of config C on one GPU: where a
# lone wave's time goes.  usage (GPU box, repo root): tools/pmc_shard.sh OUTDIR G [C]
set -o pipefail
OUT=$1; G=$2; C=${3:-c3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_IFETCH SQ_ACTIVE_INST_EXP"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d "$OUT/pass$i" -o run --output-format csv -- \
      python3 tools/shard_sweep.py --config $C --blocks 0 --strides $G --reps 5 > "$OUT/pass$i.log" 2>&1 || { echo "pass $i ($set) failed"; tail -5 "$OUT/pass$i.log"; }
done
