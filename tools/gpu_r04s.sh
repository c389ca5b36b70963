#!/bin/bash
# Round 4, final tree: the GPU suite, smoke(), the full bench line.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04s_gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -30 $O/r04s_gpu_tests.log; exit 1; }
tail -2 $O/r04s_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04s_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/r04s_smoke.log; exit 1; }
tail -1 $O/r04s_smoke.log
timeout -k 10 600 python bench.py > $O/r04s_bench.json 2> $O/r04s_bench.err || { echo BENCH_FAILED; tail -20 $O/r04s_bench.err; exit 1; }
cut -c1-300 $O/r04s_bench.json
