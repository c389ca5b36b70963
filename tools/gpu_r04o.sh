#!/bin/bash
# Round 4: flank test merged by v_alignbit (VC_FLANK_ALIGN) against the default.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
bash tools/r03_ab.sh $O/r04o_ab_fa.log "default fa" --rounds 10 || { echo AB_FAILED; tail -20 $O/r04o_ab_fa.log; exit 1; }
grep -E "^==|median|identical" $O/r04o_ab_fa.log
bash tools/gpu_r04p.sh
