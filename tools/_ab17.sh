V=$PWD/bwidman-raytracer_amd/build/variants
BWRT_LIB=$V/h20/libbwrt.so timeout -k 10 300 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "config3 or 07_small or random or quads" > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc = 0 ] || exit 1
for r in 1 2 3; do for v in base h20; do BWRT_LIB=$V/$v/libbwrt.so timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 && echo "$v $(grep -o '"ms_per_step[^,]*' gpurun_out/b.log)"; done; done
