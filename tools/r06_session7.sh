#!/bin/bash
# Round-6 GPU session 7: the HEAD profile set — config-3 PMC passes (HBM
# bytes, VALU, L1) for profiles/traffic_c3.json, rocprof kernel stats of the
# c3 and c5 benches.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06g; mkdir -p $O
timeout -k 10 500 bash tools/pmc.sh $O/pmc_c3 --config c3 --steps 3 --warmup 1 > $O/pmc_c3.log 2>&1 || exit 1
python3 tools/make_traffic_json.py $O/pmc_c3 07-1920x1080-8spp-4b-rows1 $O/traffic_c3.json > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c3 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --traffic-json $O/traffic_c3.json > $O/rocprof_c3_bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rocprof_c5 -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --config c5 --steps 5 --warmup 2 > $O/rocprof_c5_bench.log 2>&1 || exit 1
echo done > $O/done.txt
# the triangle distance skip (RT_CULL_DIST, build/variants/cd1): parity
# subset, then config 3 and its shards against HEAD
SUBSET="config3_07_full or config3_shards or random_scenes or quads or 07_small or pair_kernel_forced or global_records_forced" \
    timeout -k 10 600 bash tools/ab.sh "cd1:cd1:" > $O/parity_cd1.txt 2>&1 || exit 1
ROUNDS=3 MODE=bench timeout -k 10 400 bash tools/ab.sh "head:base:" "cd1:cd1:" > $O/ab_cd1_c3.txt 2>&1 || exit 1
ROUNDS=2 MODE=shard STRIDES=2,4,8 timeout -k 10 300 bash tools/ab.sh "head:base:" "cd1:cd1:" > $O/ab_cd1_shards.txt 2>&1 || exit 1
echo done2 > $O/done2.txt
