#!/bin/bash
# Closing measurements of a round on the GPU box (run from the repo root):
#   bench line (N = 1, defaults), bench lines for c3 and c5 (kernel only),
#   rocprofv3 --kernel-trace --stats of the C2 and C5 bench commands (full
#   passes only), PMC counters for C2 and C5 (tools/pmc.py, one pass each).
# Usage: tools/final_profile.sh TAG   -> gpurun_out/TAG_*
set -e -o pipefail
TAG=${1:?tag}
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"
timeout -k 10 400 python bench.py > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err"
timeout -k 10 300 python bench.py --config c3 --no-cpu --no-e2e > "$O/${TAG}_bench_c3.json" 2> "$O/${TAG}_bench_c3.err"
timeout -k 10 300 python bench.py --config c5 --no-cpu --no-e2e > "$O/${TAG}_bench_c5.json" 2> "$O/${TAG}_bench_c5.err"
cd /tmp
export TMPDIR=/tmp
for C in c2 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof_$C" -o p --output-format csv -- \
    python3 "$R/bench.py" --config $C --steps 10 --warmup 2 --no-parity --no-e2e --no-cpu \
    > "$O/${TAG}_prof_$C.json" 2> "$O/${TAG}_prof_$C.err"
done
cd "$R"
timeout -k 10 900 python tools/pmc.py "$O/${TAG}_pmc_c2" --steps 2 --warmup 1 --no-cpu --no-e2e --no-parity \
  > "$O/${TAG}_pmc_c2.log" 2>&1
timeout -k 10 900 python tools/pmc.py "$O/${TAG}_pmc_c5" --config c5 --steps 2 --warmup 1 --no-cpu --no-e2e --no-parity \
  > "$O/${TAG}_pmc_c5.log" 2>&1
echo done
