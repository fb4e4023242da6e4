#!/bin/bash
# Round-6 GPU session 15: RT_NT_PIXEL=1 on the shards, config 2 and 5, and
# its HBM bytes (FETCH_SIZE / WRITE_SIZE passes) against HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06r; mkdir -p $O
V=$PWD/bwidman-raytracer_amd/build/variants
for lab in head nt; do
  lib=$PWD/bwidman-raytracer_amd/lib/libbwrt.so; [ $lab = nt ] && lib=$V/nt/libbwrt.so
  for c in FETCH_SIZE WRITE_SIZE; do
    BWRT_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_${lab}_$c -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/pmc_${lab}_$c.log 2>&1 || exit 1
  done
done
ROUNDS=2 MODE=shard STRIDES=2,4,8 timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_nt_shards.txt 2>&1 || exit 1
CONFIG=c2 WARMUP=40 STEPS=40 ROUNDS=3 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_nt_c2.txt 2>&1 || exit 1
CONFIG=c5 WARMUP=2 STEPS=3 ROUNDS=2 MODE=bench timeout -k 10 600 bash tools/ab.sh "head:base:" "nt:nt:" > $O/ab_nt_c5.txt 2>&1 || exit 1
echo done > $O/done.txt
