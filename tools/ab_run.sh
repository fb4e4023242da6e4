#!/bin/bash
# one GPU A/B session (on the box, from the repo root): the rt_sqrt.h
# exhaustive check, the GPU suite (or SUBSET, a pytest -k expression) with the
# candidate library, then 5 alternating c3 and 2 c4 bench runs.
# usage: CAND=name [BASE=name] [SUBSET=expr] bash tools/ab_run.sh
# (variants from tools/variants.sh; BASE=base is lib/libbwrt.so)
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
CAND=${CAND:?set CAND to a tools/variants.sh name}; BASE=${BASE:-base}
mkdir -p gpurun_out
timeout -k 10 120 build/sqrtx || exit 1
BWRT_LIB=$V/$CAND/libbwrt.so timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread ${SUBSET:+-k "$SUBSET"} > gpurun_out/ab_pt.log 2>&1; rc=$?; tail -1 gpurun_out/ab_pt.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 tools/ab_libs.sh 5 $BASE $CAND || exit 1
BENCH_ARGS="--config c4 --steps 5 --warmup 2" timeout -k 10 300 tools/ab_libs.sh 2 $BASE $CAND
