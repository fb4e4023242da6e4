V=$PWD/bwidman-raytracer_amd/build/variants
for r in 1 2; do for v in base r32 r36 r40 r40l56 r40l60 r36l60; do echo "== $v"; BWRT_LIB=$V/$v/libbwrt.so timeout -k 10 300 python tools/shard_sweep.py --config c5 --blocks 0 --strides 1,8 --reps 3 2>&1 | grep -v amdgpu.ids; done; done
