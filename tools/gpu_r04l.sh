#!/bin/bash
# Round 4: the parallel reader's slots allocated lazily by the workers
# (default) against up front (VAFC_RESERVE=1), and 32 slots against 18, on
# the whole plain C2 stream, with the ingest profile.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 900 python tools/e2e_ab.py --rounds 6 lazy=$C,$D upfront=$C,VAFC_RESERVE=1,$D lazy32=$C,VAFC_INGEST_SLOTS=32,$D > $O/r04l_slots_ab.json 2> $O/r04l_slots_ab.err || { echo AB_FAILED; tail -20 $O/r04l_slots_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04l_slots_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)];[print(n, x[:2]) for n, x in d.get('diag', {}).items()]"
