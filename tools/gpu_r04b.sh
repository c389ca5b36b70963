#!/bin/bash
# round-4 session: GPU suite, C2 profile of the bench command, kernel A/B of lib_ab variants
set -o pipefail
R=$(pwd); O=$R/gpurun_out; TAG=${TAG:-r04b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
tail -2 $O/${TAG}_gpu_tests.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_c2 -o p --output-format csv -- python3 $R/bench.py --config c2 --steps 10 --warmup 2 --no-parity --no-e2e --no-cpu > $O/${TAG}_prof_c2.json 2> $O/${TAG}_prof_c2.err ) || { echo PROF_FAILED; exit 1; }
cat $O/${TAG}_prof_c2.json
bash tools/r03_ab.sh $O/${TAG}_ab.log "${ABVARS:-default base salu}" --rounds 10 || { echo AB_FAILED; tail -20 $O/${TAG}_ab.log; exit 1; }
grep -E "^==|median" $O/${TAG}_ab.log
