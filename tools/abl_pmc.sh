#!/bin/bash
# Ablation breakdown of the C2 kernel (k = 21 flank kernel): time per variant
# (tools/ab.py, one process) and instruction counts per variant (one
# rocprofv3 --pmc pass over the same variants).  VAFC_ABLATE: 0 full, 4 no hit
# loop, 1 no LDS filter reads, 5 = 1+4, 2 no read loads, 7 VALU only.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; TAG=${TAG:-r04c}
V="${ABL:-VAFC_ABLATE=0 VAFC_ABLATE=4 VAFC_ABLATE=1 VAFC_ABLATE=5 VAFC_ABLATE=2 VAFC_ABLATE=7}"
export VAFC_LIB=$R/kmer-cnt_amd/lib_ab/abl/libvafc.so
timeout -k 10 300 python tools/ab.py --rounds 6 $V > $O/${TAG}_abl_time.log 2>&1 || { echo ABL_TIME_FAILED; tail $O/${TAG}_abl_time.log; exit 1; }
cat $O/${TAG}_abl_time.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/${TAG}_abl_pmc -o p --output-format csv -- python3 $R/tools/ab.py --rounds 1 $V > $O/${TAG}_abl_pmc.log 2>&1 || { echo ABL_PMC_FAILED; tail $O/${TAG}_abl_pmc.log; exit 1; }
echo pmc done
