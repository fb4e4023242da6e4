run() { echo "== $*"; env "$@" timeout -k 10 300 python tools/shard_sweep.py --config c5 --blocks 0 --strides 1 --reps 3 2>&1 | grep -v amdgpu.ids; }
for r in 1 2; do
run BWRT_X=0
run BWRT_BVH_ORDER_MASK=7
run BWRT_BVH_ORDER_MASK=1
run BWRT_BVH_LEAF=4
run BWRT_BVH_LEAF=12
run BWRT_BVH_CT=2
run BWRT_BVH_CT=0.5
run BWRT_BVH_REFS=3
run BWRT_BVH_REFS=1.5
done
