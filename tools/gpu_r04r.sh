#!/bin/bash
# Round 4: gzip inflate workers (16 = -t, the default) against 14 and 13 beside
# the 3 parse workers, under the box's 16-CPU quota, on the whole gzip C2 stream.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 1000 python tools/e2e_ab.py --rounds 3 --gzip i16=$C,$D i14=$C,VAFC_GZ_INFLATERS=14,$D i13=$C,VAFC_GZ_INFLATERS=13,$D > $O/r04r_gzinflaters_ab.json 2> $O/r04r_gzinflaters_ab.err || { echo AB_FAILED; tail -20 $O/r04r_gzinflaters_ab.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04r_gzinflaters_ab.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
