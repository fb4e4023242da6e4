V=$PWD/bwidman-raytracer_amd/build/variants
BWRT_LIB=$V/pv4/libbwrt.so timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "config3 or 07 or random or quads or config2 or config4" > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc = 0 ] || exit 1
bash tools/ab_libs.sh 5 base pv4
