set -o pipefail
for v in old base; do
  L=$PWD/bwidman-raytracer_amd/build/variants/old/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
  for c in c2 c4; do
    echo "$v $c $(BWRT_LIB=$L timeout -k 10 150 python tools/shard_sweep.py --config $c --strides 1,2,8 --blocks 0 --reps 10 2>&1 | grep -o 'stride [0-9]*: median [0-9.]*' | tr '\n' ' ')" || exit 1
  done
done
