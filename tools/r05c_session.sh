set -o pipefail
export BWRT_TUNING=1
mkdir -p gpurun_out/r05c
for g in 1 4 8; do
  BWRT_LIB=$PWD/bwidman-raytracer_amd/build/variants/stamps/libbwrt.so timeout -k 10 120 python tools/stamps_run.py $g > gpurun_out/r05c/stamps_c3_$g.log 2>&1 || { tail -5 gpurun_out/r05c/stamps_c3_$g.log; exit 1; }
  echo "stride=$g $(grep stamps gpurun_out/r05c/stamps_c3_$g.log)"
done
for r in 1 2 3; do
  for sp in pol 0; do
    if [ $sp = pol ]; then E=""; else E="BWRT_SPREAD=0"; fi
    env $E timeout -k 10 120 python bench.py --config c1 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/r05c/c1_$sp.log 2>&1 || exit 1
    echo "c1 spread=$sp $(grep -o '"kernel_ms_avg[^,]*' gpurun_out/r05c/c1_$sp.log)"
  done
done
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05c/bench_c5.log 2>&1 || exit 1
tail -1 gpurun_out/r05c/bench_c5.log | cut -c1-200
bash tools/pmc_mem.sh c5 > gpurun_out/r05c/pmc_mem_c5.txt 2>&1; tail -40 gpurun_out/r05c/pmc_mem_c5.txt
