#!/bin/bash
# Round 4: gzip parse workers (3 = (16 + 3) / 5, the default) against 2 and 4
# now that the record fast path parses faster, on the whole gzip C2 stream.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 1000 python tools/e2e_ab.py --rounds 3 --gzip p3=$C,$D p2=$C,VAFC_GZ_PARSERS=2,$D p4=$C,VAFC_GZ_PARSERS=4,$D > $O/r04m_gzparsers_ab.json 2> $O/r04m_gzparsers_ab.err || { echo AB_FAILED; tail -20 $O/r04m_gzparsers_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04m_gzparsers_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)];[print(n, x[:1]) for n, x in d.get('diag', {}).items()]"
timeout -k 10 900 python tools/e2e_ab.py --rounds 5 s32=$C,$D s18=$C,VAFC_INGEST_SLOTS=18,$D > $O/r04m_slots_confirm.json 2> $O/r04m_slots_confirm.err || { echo AB2_FAILED; tail -20 $O/r04m_slots_confirm.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04m_slots_confirm.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
