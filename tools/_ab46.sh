V=$PWD/bwidman-raytracer_amd/build/variants
for r in 1 2 3; do for v in base hints; do for c in c3 c4; do echo "== $v $c"; BWRT_LIB=$V/$v/libbwrt.so timeout -k 10 200 python tools/shard_sweep.py --config $c --blocks 0 --strides 1 --reps 20 2>&1 | grep -v amdgpu.ids; done; done; done
