#!/bin/bash
set -o pipefail
R=$(pwd); O=$R/gpurun_out
bash tools/r03_ab.sh $O/r04c_ab_pf.log "default pf pp" --rounds 10 || { echo AB_FAILED; tail -20 $O/r04c_ab_pf.log; exit 1; }
grep -E "^==|median|identical" $O/r04c_ab_pf.log
bash tools/abl_pmc.sh || exit 1
timeout -k 10 600 python tools/n8_projection.py --shards 8 --runs 3 > $O/r04c_n8.json 2> $O/r04c_n8.err || { echo N8_FAILED; tail -20 $O/r04c_n8.err; exit 1; }
cat $O/r04c_n8.json
timeout -k 10 900 python tools/e2e_ab.py --rounds 4 numa=kmer-cnt_amd/lib_ab/numa/vaf-counter nonuma=kmer-cnt_amd/lib_ab/numa/vaf-counter,VAFC_NUMA=0 > $O/r04c_numa_ab.json 2> $O/r04c_numa_ab.err || { echo NUMA_AB_FAILED; tail -20 $O/r04c_numa_ab.err; exit 1; }
cat $O/r04c_numa_ab.json
