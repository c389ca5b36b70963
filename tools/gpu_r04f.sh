#!/bin/bash
# Round 4: e2e thread-count / CFS-quota study, gzip single-stream shape, then
# the closing profile (tools/final_profile_r04.sh).
set -o pipefail
R=$(pwd); O=$R/gpurun_out
cat /sys/fs/cgroup/cpu.stat > $O/r04f_cpu_stat_start.txt 2>&1
C=kmer-cnt_amd/lib/vaf-counter
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 t16=$C t14=$C,T=14 t12=$C,T=12 t16nonuma=$C,VAFC_NUMA=0 > $O/r04f_threads_ab.json 2> $O/r04f_threads_ab.err || { echo THREADS_AB_FAILED; tail -20 $O/r04f_threads_ab.err; exit 1; }
cat $O/r04f_threads_ab.json
timeout -k 10 600 python tools/e2e_ab.py --reads 20000000 --gzip-single --rounds 3 t16=$C t14=$C,T=14 > $O/r04f_gzip_single.json 2> $O/r04f_gzip_single.err || { echo GZS_FAILED; tail -20 $O/r04f_gzip_single.err; exit 1; }
cat $O/r04f_gzip_single.json
bash tools/final_profile_r04.sh r04f_final
