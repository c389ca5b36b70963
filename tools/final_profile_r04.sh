#!/bin/bash
# Round-4 closing measurements (run from the repo root on the GPU box):
# bench lines C2 (full: e2e, CPU baseline) / C3 / C4 / C5, rocprofv3 kernel
# stats of the C2 and C5 bench commands, PMC for C2 and C5.  Each step runs
# under its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r04_final}
R=$(pwd); O=$R/gpurun_out
step() { local lim=$1; shift; timeout -k 10 "$lim" "$@" || { echo "STEP FAILED ($?): $*"; exit 1; }; }
step 600 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err
cat $O/${TAG}_bench.json | cut -c1-400
step 300 python bench.py --config c5 --no-cpu --no-e2e > $O/${TAG}_bench_c5.json 2> $O/${TAG}_bench_c5.err
step 300 python bench.py --config c3 --no-cpu --no-e2e > $O/${TAG}_bench_c3.json 2> $O/${TAG}_bench_c3.err
cd /tmp && export TMPDIR=/tmp
for C in c2 c5; do
  step 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof_$C -o p --output-format csv -- \
    python3 $R/bench.py --config $C --steps 10 --warmup 2 --no-parity --no-e2e --no-cpu > $O/${TAG}_prof_$C.json 2> $O/${TAG}_prof_$C.err
  python3 $R/tools/trace_avg.py $O/${TAG}_prof_$C/p_kernel_trace.csv vc_count_reads_kernel 10 > $O/${TAG}_prof_${C}_timed.json || exit 1
done
cd $R
step 900 python tools/pmc.py $O/${TAG}_pmc_c2 --steps 2 --warmup 1 --no-cpu --no-e2e --no-parity > $O/${TAG}_pmc_c2.log 2>&1
step 900 python tools/pmc.py $O/${TAG}_pmc_c5 --config c5 --steps 2 --warmup 1 --no-cpu --no-e2e --no-parity > $O/${TAG}_pmc_c5.log 2>&1
echo done
