#!/bin/bash
# Piece-size x thread sweep of the parallel reader (vc_count_file on a plain
# FASTQ), with the reader's phase profile:
#   tools/e2e_piece_sweep.sh [n_reads] [copies]
set -e
N=${1:-4000000}; COPIES=${2:-4}
D=${TMPDIR:-/tmp}/vafc_sweep; mkdir -p $D
trap "rm -rf $D" EXIT
python - "$D" "$N" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc_synth as S
d, n = sys.argv[1], int(sys.argv[2])
p = S.grch38_panel(); p.write_patterns(d + '/pat.txt', 21)
S.write_fastq(d + '/r.fq', p, n, f_snp=0.01)
PY
for i in $(seq $COPIES); do cat $D/r.fq; done > $D/big.fq
rm $D/r.fq
cat $D/big.fq > /dev/null
for rep in 1 2; do
for T in 4 8 16; do
for P in 8388608 16777216; do
  VAFC_INGEST_PROFILE=1 VAFC_INGEST_PIECE=$P timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -t $T -p $D/pat.txt -o $D/o.vaf $D/big.fq 2> $D/e.err
  echo "rep $rep piece $P -t $T: $(grep Speed $D/e.err | sed 's/ \+/ /g') $(grep ingest $D/e.err)"
done
done
done
