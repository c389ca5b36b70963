#!/bin/bash
# End-to-end rate of the drop-in CLI on gzip FASTQ (what sequencers deliver):
# the parallel inflater (vafc_gzip.cpp) with -t 1/4/16 workers vs the
# reference binary (oracle/_ref, one zlib stream) on the same files; the .vaf
# files must be identical.  Also the host-only ceiling (inflate + kseq parse
# + block loop, no device).
#   tools/e2e_gz.sh [n_reads] [k]
set -e
N=${1:-4000000}; K=${2:-21}
D=${TMPDIR:-/tmp}/vafc_e2e_gz; mkdir -p $D
trap "rm -rf $D" EXIT
python - "$D" "$N" "$K" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc_synth as S
d, n, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
p = S.grch38_panel(); p.write_patterns(d + '/pat.txt', k)
S.write_fastq(d + '/r.fq', p, n, f_snp=0.01)
S.write_fastq(d + '/s.fq', p, n // 4, seed=43, f_snp=0.01)
PY
t0=$(date +%s.%N); gzip -1 -c $D/r.fq > $D/r1.fq.gz; t1=$(date +%s.%N)
gzip -6 -c $D/s.fq > $D/s6.fq.gz; t2=$(date +%s.%N)
echo "gzip -1: $(stat -c %s $D/r.fq) -> $(stat -c %s $D/r1.fq.gz) bytes ($(python -c "print(round($t1-$t0,1))") s); gzip -6: $(stat -c %s $D/s.fq) -> $(stat -c %s $D/s6.fq.gz) bytes ($(python -c "print(round($t2-$t1,1))") s)"
cat $D/r1.fq.gz $D/s6.fq.gz > /dev/null

for F in s6 r1; do
  for T in 1 4 16 16; do
    timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -t $T -k $K -p $D/pat.txt -o $D/gpu_${F}_t$T.vaf $D/$F.fq.gz 2> $D/gpu_${F}_t$T.err
    grep -E "Speed" $D/gpu_${F}_t$T.err | sed "s/^/gpu $F.fq.gz -t$T: /"
  done
  echo "vaf identical across -t ($F): $(cmp -s $D/gpu_${F}_t1.vaf $D/gpu_${F}_t4.vaf && cmp -s $D/gpu_${F}_t1.vaf $D/gpu_${F}_t16.vaf && echo yes || echo NO)"
done
timeout -k 10 600 oracle/_ref/vaf-counter -v -t 1 -k $K -p $D/pat.txt -o $D/ref_s6.vaf $D/s6.fq.gz 2> $D/ref_s6.err
grep -E "Speed" $D/ref_s6.err | sed "s/^/ref s6.fq.gz -t1: /"
echo "vaf identical to the reference (s6): $(cmp -s $D/gpu_s6_t16.vaf $D/ref_s6.vaf && echo yes || echo NO)"

VAFC_GZ_PROFILE=1 python - "$D/r1.fq.gz" "$D/s6.fq.gz" "$K" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc
k = int(sys.argv[3])
for fn in sys.argv[1:3]:
    for t in (4, 16):
        st, _ = vafc.scan_file_parallel(fn, k, threads=t, piece_bytes=4 << 20)
        print("host ingest only, %s, %d inflate workers: %.0f Mbases/s (%.0f MB/s of FASTQ)"
              % (fn.split('/')[-1], t, st.bases / st.seconds / 1e6, st.bases / st.seconds / 1e6 * 311 / 150))
PY
