timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -1 gpurun_out/pt.log; [ $rc = 0 ] || { grep -E "FAIL|Error" gpurun_out/pt.log | head; exit 1; }
bash tools/ab_libs.sh 5 base nq2
