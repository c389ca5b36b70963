#!/bin/bash
# End-to-end (PCIe-inclusive) rate of the drop-in CLI on the GPU box: a
# synthetic FASTQ in page cache, the HIP vaf-counter vs the reference binary
# (oracle/_ref, built here from /root/reference) on the same file.  Prints the
# -v "Speed" lines and checks the two .vaf files are identical.
#   tools/e2e.sh [n_reads] [k]
set -e
N=${1:-4000000}; K=${2:-21}
D=${TMPDIR:-/tmp}/vafc_e2e; mkdir -p $D
trap "rm -rf $D" EXIT
python - "$D" "$N" "$K" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc_synth as S
d, n, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
p = S.grch38_panel(); p.write_patterns(d + '/pat.txt', k)
S.write_fastq(d + '/r.fq', p, n, f_snp=0.01)
PY
cat $D/r.fq > /dev/null
for rep in 1 2; do
  timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -k $K -p $D/pat.txt -o $D/gpu.vaf $D/r.fq 2> $D/gpu.err
  grep -E "Speed|Time|K-mers extracted" $D/gpu.err | sed "s/^/gpu rep$rep: /"
done
timeout -k 10 600 oracle/_ref/vaf-counter -v -t 1 -k $K -p $D/pat.txt -o $D/ref.vaf $D/r.fq 2> $D/ref.err
grep -E "Speed|Time|K-mers extracted" $D/ref.err | sed "s/^/ref -t1: /"
echo "vaf identical: $(cmp -s $D/gpu.vaf $D/ref.vaf && echo yes || echo NO)"
# host-only ingest (reader + block loop, no device): the ceiling of the CLI
python - "$D/r.fq" "$K" <<'PY'
import sys, time; sys.path.insert(0, 'kmer-cnt_amd')
import vafc
fn, k = sys.argv[1], int(sys.argv[2])
st = vafc.scan_file(fn, k)
st = st[0] if isinstance(st, tuple) else st
print("host ingest only (plain): %.0f Mbases/s" % (st.bases / st.seconds / 1e6))
PY
# gzip input (what sequencers deliver): zlib inflate bounds both programs
gzip -1 -c $D/r.fq > $D/r.fq.gz
timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -k $K -p $D/pat.txt -o $D/gpu_gz.vaf $D/r.fq.gz 2> $D/gpu_gz.err
grep -E "Speed" $D/gpu_gz.err | sed "s/^/gpu gz: /"
timeout -k 10 600 oracle/_ref/vaf-counter -v -t 1 -k $K -p $D/pat.txt -o $D/ref_gz.vaf $D/r.fq.gz 2> $D/ref_gz.err
grep -E "Speed" $D/ref_gz.err | sed "s/^/ref gz -t1: /"
echo "gz vaf identical: $(cmp -s $D/gpu_gz.vaf $D/ref_gz.vaf && echo yes || echo NO)"
