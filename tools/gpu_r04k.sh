#!/bin/bash
# Round 4: pinned-slot allocation cost, and the vectorised newline scan of
# the reader's fast path against memchr on the whole C2 stream.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 120 ./tools/alloc_probe > $O/r04k_alloc_probe.log 2>&1 || { echo ALLOC_PROBE_FAILED; cat $O/r04k_alloc_probe.log; exit 1; }
cat $O/r04k_alloc_probe.log
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 vector=$C,$D memchr=$C,VAFC_NL_SCAN=memchr,$D > $O/r04k_nlscan_ab.json 2> $O/r04k_nlscan_ab.err || { echo AB_FAILED; tail -20 $O/r04k_nlscan_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04k_nlscan_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)];[print(n, x[:1]) for n, x in d.get('diag', {}).items()]"
