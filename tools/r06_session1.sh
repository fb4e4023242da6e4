#!/bin/bash
# Round-6 GPU session 1 (run on the GPU box from the repo root):
# RCCL path at world 1, the 8-wave global-record shape (parity + shard A/B),
# the L1 micro-benchmark, the c3 stamps split at HEAD, the c5 coherent-wave
# experiment.  Every GPU step has its own time limit; the first failure ends
# the session.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06a; mkdir -p $O
step() { echo "== $(date +%T) $1" | tee -a $O/steps.txt; }
step rccl-test
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > $O/pt_bench.log 2>&1 || exit 1
step rccl-bench
NCCL_DEBUG=INFO timeout -k 10 200 python bench.py --gpus 1 --dist --steps 20 --warmup 5 > $O/dist1.log 2>&1 || exit 1
step grec-parity
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "global_records_forced or config3_shards or config3_07_full" > $O/pt_grec.log 2>&1 || exit 1
step grec-ab
ROUNDS=2 MODE=shard STRIDES=1,2,3,4 REPS=20 timeout -k 10 300 bash tools/ab.sh "pol:base:" "g0:base:BWRT_GREC=0" \
    "g1:base:BWRT_GREC=1" "g2:base:BWRT_GREC=2" > $O/ab_grec.txt 2>&1 || exit 1
cp gpurun_out/ab/s_*.log $O/ 2>/dev/null
step micro
timeout -k 10 120 build/ta_gather > $O/ta_gather_micro.txt 2>&1 || exit 1
step stamps
BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/stamps/libbwrt.so timeout -k 10 120 python tools/stamps_run.py 1 2 4 8 \
    > $O/stamps_c3.log 2>&1 || exit 1
step coherent
SUBSET="stress_scene_small or stress_c5_rows_bvh or config5_rows_32spp or bvh_refill_schedules" \
CANDS="refill: c0_256:BWRT_BVH_SORTED=1,BWRT_BVH_BLOCK=256 c1_256:BWRT_BVH_SORTED=2,BWRT_BVH_BLOCK=256 c2_256:BWRT_BVH_SORTED=3,BWRT_BVH_BLOCK=256 c0_1024:BWRT_BVH_SORTED=1,BWRT_BVH_BLOCK=1024 c2_1024:BWRT_BVH_SORTED=3,BWRT_BVH_BLOCK=1024" \
    timeout -k 10 600 bash tools/c5_coherent_ab.sh > $O/coherent.txt 2>&1 || exit 1
step done
