#!/bin/bash
# Round 4: plain e2e, one-line sequences in place vs copied (VAFC_SEQ_INPLACE=0),
# with the ingest profile, and the reader alone.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 --host-parse inplace=$C,$D copy=$C,VAFC_SEQ_INPLACE=0,$D > $O/r04h_inplace_ab.json 2> $O/r04h_inplace_ab.err || { echo AB_FAILED; tail -20 $O/r04h_inplace_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04h_inplace_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)];[print(n, x[:1]) for n, x in d.get('diag', {}).items()]"
