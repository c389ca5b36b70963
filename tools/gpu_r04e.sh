#!/bin/bash
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/r04e_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/r04e_gpu_tests.log; exit 1; }
tail -2 $O/r04e_gpu_tests.log
bash tools/gpu_r04d.sh
