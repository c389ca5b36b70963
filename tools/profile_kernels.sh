#!/bin/bash
# Kernel profiles on the GPU box (run from the repo root):
#   tools/profile_kernels.sh TAG [CONFIG...]   (default configs: c2 c5)
# per config: rocprofv3 --kernel-trace --stats of bench.py's own command
# (kernel only: no parity sample, no e2e leg, no CPU baseline) and the PMC
# passes of tools/pmc.py (one rocprofv3 --pmc run per counter group).
# Outputs: gpurun_out/TAG_prof_C/ (stats CSV), gpurun_out/TAG_pmc_C/.
set -e -o pipefail
TAG=${1:?tag}
shift
CONFIGS=${*:-c2 c5}
R=$(pwd)
O=$R/gpurun_out
mkdir -p "$O"
for C in $CONFIGS; do
  cd /tmp
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof_$C" -o p --output-format csv -- \
    python3 "$R/bench.py" --config $C --steps 10 --warmup 2 --no-parity --no-e2e --no-cpu \
    > "$O/${TAG}_prof_$C.json" 2> "$O/${TAG}_prof_$C.err"
  cd "$R"
  timeout -k 10 900 python tools/pmc.py "$O/${TAG}_pmc_$C" --config $C --steps 2 --warmup 1 --no-cpu --no-e2e \
    --no-parity > "$O/${TAG}_pmc_$C.log" 2>&1
done
echo done
