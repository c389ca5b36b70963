#!/bin/bash
# Round 4: the C4 bench line (1B reads on one GPU) on the final tree.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 600 python bench.py --config c4 --no-cpu --no-e2e > $O/r04v_bench_c4.json 2> $O/r04v_bench_c4.err || { echo BENCH_FAILED; tail -20 $O/r04v_bench_c4.err; exit 1; }
cut -c1-400 $O/r04v_bench_c4.json
