#!/bin/bash
# Per-phase VALU instructions and lane-cycles of the c3 sorted kernel: PMC
# (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU, SQ_WAVES) of the plain library and of
# the RT_PHASE_TWICE = 1..4 variants (closest hit / RANDDIR / SPEC / fold run
# twice; build them first: tools/variants.sh ph1 -DRT_PHASE_TWICE=1 ...), one
# pass each; tools/phase_lanes.py turns the deltas into the breakdown.
# usage (GPU box, repo root): tools/phase_lanes.sh OUTDIR [bench args]
set -o pipefail
export BWRT_TUNING=1
OUT=$1; shift
V=$PWD/bwidman-raytracer_amd/build/variants
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p "$OUT"
for v in base ph1 ph2 ph3 ph4; do
  L=$V/$v/libbwrt.so; [ $v = base ] && L=$PWD/bwidman-raytracer_amd/lib/libbwrt.so
  BWRT_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES \
      -d "$OUT/$v" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 5 --warmup 1 "$@" \
      > "$OUT/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.log"; exit 1; }
  echo "$v done"
done
python3 tools/phase_lanes.py "$OUT"
