V=$PWD/bwidman-raytracer_amd/build/variants
BWRT_LIB=$V/t24/libbwrt.so timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "config3 or 07 or random or quads or config2 or config4 or shard or ragged or bounce" > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc = 0 ] || { grep -E "FAIL|Error" gpurun_out/pt.log | head; exit 1; }
for r in 1 2; do for v in base t4 t12 t24; do echo "== $v"; BWRT_LIB=$V/$v/libbwrt.so timeout -k 10 200 python tools/shard_sweep.py --blocks 0 --strides 1,2,4,8 --reps 20 2>&1 | grep -v amdgpu.ids; done; done
