#!/bin/bash
# Round 4: the compiler's scheduling strategy for the counting kernel
# (max-ilp, iterative-ilp) against the default, C2 and C5.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
bash tools/r03_ab.sh $O/r04u_ab_sched_c2.log "default milp iilp" --rounds 10 || { echo AB_FAILED; tail -20 $O/r04u_ab_sched_c2.log; exit 1; }
grep -E "^==|median|identical" $O/r04u_ab_sched_c2.log
bash tools/r03_ab.sh $O/r04u_ab_sched_c5.log "default milp iilp" --rounds 6 --panel syn200k || { echo AB5_FAILED; tail -20 $O/r04u_ab_sched_c5.log; exit 1; }
grep -E "^==|median|identical" $O/r04u_ab_sched_c5.log
