#!/bin/bash
# Round 4 closing call: the GPU suite, smoke(), then the closing profile.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04j_gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -30 $O/r04j_gpu_tests.log; exit 1; }
tail -2 $O/r04j_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04j_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/r04j_smoke.log; exit 1; }
tail -2 $O/r04j_smoke.log
bash tools/final_profile_r04.sh r04j_final
