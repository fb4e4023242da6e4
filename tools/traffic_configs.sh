#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) for the non-headline bench
# configs, then their bench lines with `roofline.traffic` filled in.
# Run on the GPU box from the repo root: tools/traffic_configs.sh c4 c5
set -o pipefail
R=$GRAFT_REPO_ROOT
for c in "$@"; do
  case $c in
    c4) key=07-3840x2160-16spp-6b-rows1 ;;
    c5) key=stress-1920x1080-32spp-8b-rows1 ;;
    *) echo "unknown config $c"; exit 1 ;;
  esac
  out=$R/gpurun_out/pmc_$c; mkdir -p $out
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    (cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set -d "$out/pass$i" -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline --config $c --steps 3 --warmup 1 > "$out/pass$i.log" 2>&1) || { echo "$c pass $i failed"; tail -5 "$out/pass$i.log"; exit 1; }
  done
  python3 tools/make_traffic_json.py $out $key $R/gpurun_out/traffic_$c.json > /dev/null || exit 1
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --config $c --steps 3 --warmup 1 \
      --traffic-json $R/gpurun_out/traffic_$c.json > $R/gpurun_out/bench_$c.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/bench_$c.log > $R/gpurun_out/bench_$c.json
  echo "$c: $(grep -o '"traffic": [0-9a-z]*' $R/gpurun_out/bench_$c.json)"
done
