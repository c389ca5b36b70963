#!/bin/bash
# Round 4: the other gzip file shapes on the final reader: one deflate stream
# (gzip -1) and BGZF (bgzip's independent 64 KiB members), 20M reads each.
set -o pipefail
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python tools/ab.py --panel syn200k --rounds 6 VAFC_L2F_BITS_PER_KEY=40 VAFC_L2F_BITS_PER_KEY=20 VAFC_L2F_BITS_PER_KEY=10 > $O/r04p_c5_l2f_size.log 2>&1 || { echo L2F_AB_FAILED; tail -20 $O/r04p_c5_l2f_size.log; exit 1; }
grep -E "median|identical" $O/r04p_c5_l2f_size.log
C=kmer-cnt_amd/lib/vaf-counter
D=VAFC_INGEST_PROFILE=1,VAFC_PHASES=1
timeout -k 10 600 python tools/e2e_ab.py --reads 20000000 --gzip-single --rounds 3 t16=$C,$D > $O/r04p_gzip_single.json 2> $O/r04p_gzip_single.err || { echo GZS_FAILED; tail -20 $O/r04p_gzip_single.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04p_gzip_single.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
timeout -k 10 600 python tools/e2e_ab.py --reads 20000000 --bgzf --rounds 3 t16=$C,$D > $O/r04p_bgzf.json 2> $O/r04p_bgzf.err || { echo BGZF_FAILED; tail -20 $O/r04p_bgzf.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04p_bgzf.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
timeout -k 10 600 python tools/e2e_ab.py --reads 20000000 --gzip --rounds 3 t16=$C,$D > $O/r04p_pigz20m.json 2> $O/r04p_pigz20m.err || { echo PIGZ_FAILED; tail -20 $O/r04p_pigz20m.err; exit 1; }
python -c "import json;d=json.load(open('$O/r04p_pigz20m.json'));[print(k, d[k]) for k in d if k not in ('diag',)]"
