set -o pipefail
V=$PWD/bwidman-raytracer_amd/build/variants
mkdir -p gpurun_out
BWRT_LIB=$V/bop/libbwrt.so timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "config3 or random or small or stress_c5" > gpurun_out/ab1_pt.log 2>&1; rc=$?; tail -1 gpurun_out/ab1_pt.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 tools/ab_libs.sh 5 old bop || exit 1
BENCH_ARGS="--config c4 --steps 5 --warmup 2" timeout -k 10 300 tools/ab_libs.sh 2 old bop
