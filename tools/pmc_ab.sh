#!/bin/bash
# PMC A/B of the render kernel: tools/_pmc_ab.sh "ENV=.. |label" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for cfg in "$@"; do
  envs=${cfg%%|*}; label=${cfg##*|}
  env $envs timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY -d gpurun_out/pmc_$label/pass1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/pmc_$label.log 2>&1 || { echo "pmc $label failed"; tail -3 gpurun_out/pmc_$label.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/pmc_$label > gpurun_out/pmc_$label.json 2>&1 || cat tools/pmc_summary.py | head -5
  echo "== $label"; cat gpurun_out/pmc_$label.json
done
