#!/bin/bash
set -e -o pipefail
R=$(pwd); O=$R/gpurun_out; cd /tmp; export TMPDIR=/tmp
for V in new prepeel; do
  if [ $V = prepeel ]; then export VAFC_LIB=$R/kmer-cnt_amd/lib_ab/libvafc_prepeel.so; fi
  for C in c5 c2; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d $O/r02_icache_${V}_$C -o p --output-format csv -- python3 $R/bench.py --config $C --steps 2 --warmup 1 --no-cpu --no-e2e --no-parity > $O/r02_icache_${V}_$C.log 2>&1
  done
done
echo ok
