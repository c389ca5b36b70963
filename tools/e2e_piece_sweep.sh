#!/bin/bash
# Piece-size sweep of the parallel reader (vc_count_file on a plain FASTQ):
#   tools/e2e_piece_sweep.sh [n_reads] [copies] [threads]
set -e
N=${1:-4000000}; COPIES=${2:-4}; T=${3:-16}
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
for P in 8388608 16777216 33554432 67108864 8388608; do
  VAFC_INGEST_PROFILE=1 VAFC_INGEST_PIECE=$P timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -t $T -p $D/pat.txt -o $D/o_$P.vaf $D/big.fq 2> $D/e_$P.err
  echo "piece $P -t $T: $(grep Speed $D/e_$P.err) $(grep ingest $D/e_$P.err)"
done
