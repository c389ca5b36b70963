set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/r04a_gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $O/r04a_gpu_tests.log; exit 1; }
tail -3 $O/r04a_gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04a_prof_c2 -o p --output-format csv -- python3 $R/bench.py --config c2 --steps 10 --warmup 2 --no-parity --no-e2e --no-cpu > $O/r04a_prof_c2.json 2> $O/r04a_prof_c2.err
cat $O/r04a_prof_c2.json
