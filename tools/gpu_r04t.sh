#!/bin/bash
# Round 4 final: GPU suite and smoke, the newline-scan A/B with the CPU model
# initialised, and the bench line.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r04t_gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -30 $O/r04t_gpu_tests.log; exit 1; }
tail -1 $O/r04t_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r04t_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 $O/r04t_smoke.log; exit 1; }
tail -1 $O/r04t_smoke.log
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 vector=$C,$D memchr=$C,VAFC_NL_SCAN=memchr,$D > $O/r04t_nlscan_ab.json 2> $O/r04t_nlscan_ab.err || { echo AB_FAILED; tail -20 $O/r04t_nlscan_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04t_nlscan_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
timeout -k 10 600 python bench.py > $O/r04t_bench.json 2> $O/r04t_bench.err || { echo BENCH_FAILED; tail -20 $O/r04t_bench.err; exit 1; }
cut -c1-200 $O/r04t_bench.json
