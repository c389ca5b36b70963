#!/bin/bash
# Kernel A/B on the GPU box: the default library against build-time variants
# (tools/ab_libs.sh, or an older commit's build in kmer-cnt_amd/lib_ab/NAME),
# same reads, alternating order, two rounds.
#   tools/r03_ab.sh OUTFILE "VARIANTS" [ab.py args...]    e.g. "default prev r2"
set -e -o pipefail
OUT=${1:?out}
VARS=${2:-default prev}
shift 2 || shift
for rep in 1 2; do
  for v in $VARS; do
    if [ "$v" = default ]; then L=kmer-cnt_amd/lib/libvafc.so; else L=kmer-cnt_amd/lib_ab/$v/libvafc.so; fi
    echo "== $v (rep $rep)" >> "$OUT"
    VAFC_LIB=$L timeout -k 10 120 python tools/ab.py "$@" VAFC_VARIANT=0 >> "$OUT" 2>&1
  done
done
