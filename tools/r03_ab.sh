#!/bin/bash
# Round-3 kernel A/B on the GPU box: the default library against the
# build-time variants of tools/ab_libs.sh, same reads, alternating order.
#   tools/r03_ab.sh OUTFILE [ab.py args...]
set -e -o pipefail
OUT=${1:?out}
shift
for rep in 1 2; do
  for v in default fb r2; do
    if [ "$v" = default ]; then L=kmer-cnt_amd/lib/libvafc.so; else L=kmer-cnt_amd/lib_ab/$v/libvafc.so; fi
    echo "== $v (rep $rep)" >> "$OUT"
    if [ "$v" = default ]; then
      VAFC_LIB=$L timeout -k 10 120 python tools/ab.py "$@" VAFC_VARIANT=0 VAFC_VARIANT=256 >> "$OUT" 2>&1
    else
      VAFC_LIB=$L timeout -k 10 120 python tools/ab.py "$@" VAFC_VARIANT=0 >> "$OUT" 2>&1
    fi
  done
done
