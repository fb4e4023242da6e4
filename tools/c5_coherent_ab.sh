#!/bin/bash
# Config 5: the coherent-wave BVH kernel (BWRT_BVH_SORTED=k, rays regrouped
# across a BWRT_BVH_BLOCK-lane group each round, sort key k-1) against the
# ray-refill kernel — parity subset, kernel times, and one PMC pass per
# candidate (L1 tag accesses, L1->L2 requests).  Run on the GPU box from the
# repo root: tools/c5_coherent_ab.sh  -> gpurun_out/coh/
# (round 6: the coherent-wave kernel lost 2.2x and was removed from the
# source; to rerun, apply profiles/r06a/coherent_kernel.diff first)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export BWRT_TUNING=1
OUT=gpurun_out/coh; mkdir -p $OUT
CANDS=${CANDS:-"refill: c0_256:BWRT_BVH_SORTED=1,BWRT_BVH_BLOCK=256 c1_256:BWRT_BVH_SORTED=2,BWRT_BVH_BLOCK=256 c2_256:BWRT_BVH_SORTED=3,BWRT_BVH_BLOCK=256 c0_1024:BWRT_BVH_SORTED=1,BWRT_BVH_BLOCK=1024 c2_1024:BWRT_BVH_SORTED=3,BWRT_BVH_BLOCK=1024"}
if [ -n "$SUBSET" ]; then
  for spec in $CANDS; do
    label=${spec%%:*}; envs=${spec#*:}
    [ -z "$envs" ] && continue
    env BWRT_LIB=$PWD/bwidman-raytracer_amd/lib/libbwrt.so BWRT_AB_ENV="$envs" timeout -k 10 600 python -u -m pytest tests -q -m gpu -x \
        --timeout 120 --timeout-method thread -k "$SUBSET" > $OUT/pt_$label.log 2>&1 || { echo "$label parity FAILED"; tail -5 $OUT/pt_$label.log; exit 1; }
    echo "$label parity: $(tail -1 $OUT/pt_$label.log)"
  done
fi
for r in $(seq ${ROUNDS:-2}); do
  for spec in $CANDS; do
    label=${spec%%:*}; envs=${spec#*:}
    env ${envs//,/ } timeout -k 10 200 python bench.py --no-cpu-baseline --config ${CONFIG:-c5} --steps ${STEPS:-5} --warmup 2 \
        > $OUT/b_$label.log 2>&1 || { echo "$label failed"; tail -3 $OUT/b_$label.log; exit 1; }
    echo "$label $(grep -o '"kernel_ms_avg[^,]*' $OUT/b_$label.log) $(grep -o '"kernel": "[^"]*' $OUT/b_$label.log)"
  done
done
[ -n "$NOPMC" ] && exit 0
for spec in $CANDS; do
  label=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
      SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU \
      -d $OUT/pmc_$label -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --config ${CONFIG:-c5} --steps 1 --warmup 1 > $OUT/pmc_$label.log 2>&1 \
      || { echo "$label pmc failed"; tail -3 $OUT/pmc_$label.log; exit 1; }
  echo "pmc $label done"
done
