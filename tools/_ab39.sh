V=$PWD/bwidman-raytracer_amd/build/variants
BWRT_LIB=$V/lp/libbwrt.so timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "stress or bvh or random" > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc = 0 ] || exit 1
for r in 1 2; do for v in base lp; do echo "== $v"; BWRT_LIB=$V/$v/libbwrt.so timeout -k 10 300 python tools/shard_sweep.py --config c5 --blocks 0 --strides 1,8 --reps 3 2>&1 | grep -v amdgpu.ids; done; done
