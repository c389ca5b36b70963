#!/bin/bash
# Round 4: the whole-record FASTQ fast path of the reader (VAFC_SEQ_INPLACE=0
# turns it off) on the plain and the gzip C2 stream, with the ingest profile.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 --host-parse fast=$C,$D bytewise=$C,VAFC_SEQ_INPLACE=0,$D > $O/r04i_fastpath_plain.json 2> $O/r04i_fastpath_plain.err || { echo AB_FAILED; tail -20 $O/r04i_fastpath_plain.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04i_fastpath_plain.json'));[print(k, d[k]) for k in d if k not in ('diag',)];[print(n, x[:1]) for n, x in d.get('diag', {}).items()]"
timeout -k 10 900 python tools/e2e_ab.py --rounds 3 --gzip fast=$C,$D bytewise=$C,VAFC_SEQ_INPLACE=0,$D > $O/r04i_fastpath_gzip.json 2> $O/r04i_fastpath_gzip.err || { echo GZ_AB_FAILED; tail -20 $O/r04i_fastpath_gzip.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04i_fastpath_gzip.json'));[print(k, d[k]) for k in d if k not in ('diag',)];[print(n, x[:1]) for n, x in d.get('diag', {}).items()]"
