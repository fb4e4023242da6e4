timeout -k 10 400 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -k "stress or bvh or random" > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
echo "== policy"; timeout -k 10 300 python tools/shard_sweep.py --config c5 --blocks 0 --strides 1,4,8 --reps 3 2>&1 | grep -v amdgpu.ids
for b in 58 60 62 63 64; do echo "== $b"; BWRT_LEAF_BATCH=$b timeout -k 10 300 python tools/shard_sweep.py --config c5 --blocks 0 --strides 4,8 --reps 3 2>&1 | grep -v amdgpu.ids; done
done
