#!/bin/bash
# Round 4: rocprofv3 kernel + memory-copy trace of the CLI on the whole plain C2 stream.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 900 python tools/e2e_prof.py $O/r04q_e2e_prof > $O/r04q_e2e_prof.log 2>&1 || { echo E2E_PROF_FAILED; tail -30 $O/r04q_e2e_prof.log; exit 1; }
cat $O/r04q_e2e_prof.log
bash tools/gpu_r04r.sh
