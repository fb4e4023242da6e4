run() { echo "== $*"; env "$@" timeout -k 10 300 python tools/shard_sweep.py --config c5 --blocks 0 --strides 1,8 --reps 3 2>&1 | grep -v amdgpu.ids; }
for r in 1 2; do
run BWRT_X=0
run BWRT_TILE=16
run BWRT_TILE=4
run BWRT_TILE=32
run BWRT_BVH_ORDER_MASK=7
done
