export BWRT_TUNING=1
set -o pipefail
for r in 1 2; do for sp in 0 1; do
BWRT_SPREAD=$sp timeout -k 10 150 python tools/shard_sweep.py --config c3 --strides 2,3,4,6 --blocks 0 --reps 20 2>&1 | grep stride | sed "s/^/spread=$sp /" || exit 1
BWRT_SPREAD=$sp timeout -k 10 150 python tools/shard_sweep.py --config c4 --strides 8,16,32 --blocks 0 --reps 10 2>&1 | grep stride | sed "s/^/spread=$sp /" || exit 1
done; done
