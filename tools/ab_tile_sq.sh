#!/bin/bash
# 2 x 2 tile groups (BWRT_TILE_SQ=1: the 4 waves of a 256-lane group as a
# square patch of 8 x 8 tiles) vs tiles in a row: GPU parity suite under the
# option, then alternating benches of configs 3, 2 and 4.
export BWRT_TUNING=1  # the library reads BWRT_* knobs only under it
set -o pipefail
mkdir -p gpurun_out/sq
BWRT_TILE_SQ=1 timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/sq/pytest_sq.log 2>&1; rc=$?; tail -1 gpurun_out/sq/pytest_sq.log; [ $rc = 0 ] || exit 1
ROUNDS=3 STEPS=50 CONFIG=c3 bash tools/ab_env.sh "t8:base:" "sq:base:BWRT_TILE_SQ=1" "t16:base:BWRT_TILE=16" "t16sq:base:BWRT_TILE=16,BWRT_TILE_SQ=1" || exit 1
ROUNDS=2 STEPS=20 CONFIG=c2 bash tools/ab_env.sh "t8:base:" "sq:base:BWRT_TILE_SQ=1" || exit 1
ROUNDS=2 STEPS=10 CONFIG=c4 bash tools/ab_env.sh "t8:base:" "sq:base:BWRT_TILE_SQ=1" || exit 1
