#!/bin/bash
set -o pipefail
R=$(pwd); O=$R/gpurun_out
cat /proc/self/cgroup > $O/r04d_cgroup.txt 2>&1; cat /sys/fs/cgroup/cpu.max >> $O/r04d_cgroup.txt 2>&1; nproc >> $O/r04d_cgroup.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/r04d_cgroup.txt
bash tools/r03_ab.sh $O/r04d_ab_hb.log "default hb fs" --rounds 10 || { echo AB_FAILED; tail -20 $O/r04d_ab_hb.log; exit 1; }
grep -E "^==|median|identical" $O/r04d_ab_hb.log
bash tools/r03_ab.sh $O/r04d_ab_c5.log "default ba2 hb" --rounds 6 --panel syn200k || { echo AB5_FAILED; tail -20 $O/r04d_ab_c5.log; exit 1; }
grep -E "^==|median|identical" $O/r04d_ab_c5.log
timeout -k 10 900 python tools/e2e_ab.py --rounds 6 numa=kmer-cnt_amd/lib/vaf-counter nonuma=kmer-cnt_amd/lib/vaf-counter,VAFC_NUMA=0 > $O/r04d_numa_ab.json 2> $O/r04d_numa_ab.err || { echo NUMA_AB_FAILED; tail -20 $O/r04d_numa_ab.err; exit 1; }
cat $O/r04d_numa_ab.json
