#!/bin/bash
# Round 4: plain e2e with the mapped-file reader against pread, with the
# ingest profile and the counting-phase split, and the reader alone.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 --host-parse mm=$C,$D pread=$C,VAFC_MMAP=0,$D > $O/r04g_mmap_ab.json 2> $O/r04g_mmap_ab.err || { echo MMAP_AB_FAILED; tail -20 $O/r04g_mmap_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04g_mmap_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
