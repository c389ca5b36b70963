#!/bin/bash
# Build-time A/B variants of libvafc.so (tools only; never shipped):
#   kmer-cnt_amd/lib_ab/<name>/libvafc.so built with XFLAGS, e.g.
#   tools/ab_libs.sh fb="-DVC_SCAN_BWD" r2="-DVC_FLANK_WORD"
# then on the GPU box: VAFC_LIB=kmer-cnt_amd/lib_ab/fb/libvafc.so python tools/ab.py VAFC_VARIANT=0
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  name=${spec%%=*}
  flags=${spec#*=}
  make -s -j8 -C "$ROOT/kmer-cnt_amd/csrc" OUT="../lib_ab/$name" XFLAGS="$flags" "../lib_ab/$name/libvafc.so"
  echo "built lib_ab/$name ($flags)"
done
