#!/bin/bash
# End-to-end (PCIe-inclusive) rate of the drop-in CLI on the GPU box: a
# synthetic FASTQ in page cache, the HIP vaf-counter vs the reference binary
# (oracle/_ref, built here from /root/reference) on the same file.  Prints the
# -v "Speed" lines and checks the .vaf files are identical.
#   tools/e2e.sh [n_reads] [k] [copies]
# The big file is `copies` back-to-back copies of the n_reads file (same
# records repeated: the counts scale, the reader and kernels do the same work).
set -e
N=${1:-4000000}; K=${2:-21}; COPIES=${3:-4}
D=${TMPDIR:-/tmp}/vafc_e2e; mkdir -p $D
trap "rm -rf $D" EXIT
python - "$D" "$N" "$K" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc_synth as S
d, n, k = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
p = S.grch38_panel(); p.write_patterns(d + '/pat.txt', k)
S.write_fastq(d + '/r.fq', p, n, f_snp=0.01)
PY
for i in $(seq $COPIES); do cat $D/r.fq; done > $D/big.fq
cat $D/r.fq $D/big.fq > /dev/null
echo "small file: $N reads, $(stat -c %s $D/r.fq) bytes; big file: $COPIES copies, $(stat -c %s $D/big.fq) bytes"

# parity on the small file: GPU CLI (parallel reader, default -t 4) vs reference
timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -k $K -p $D/pat.txt -o $D/gpu.vaf $D/r.fq 2> $D/gpu.err
grep -E "Speed|K-mers extracted" $D/gpu.err | sed "s/^/gpu small -t4: /"
timeout -k 10 600 oracle/_ref/vaf-counter -v -t 1 -k $K -p $D/pat.txt -o $D/ref.vaf $D/r.fq 2> $D/ref.err
grep -E "Speed|K-mers extracted" $D/ref.err | sed "s/^/ref small -t1: /"
echo "vaf identical (small): $(cmp -s $D/gpu.vaf $D/ref.vaf && echo yes || echo NO)"

# the big file with 1, 4 and 16 reader threads; all .vaf identical
for T in 1 4 16 16; do
  timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -t $T -k $K -p $D/pat.txt -o $D/gpu_t$T.vaf $D/big.fq 2> $D/gpu_t$T.err
  grep -E "Speed" $D/gpu_t$T.err | sed "s/^/gpu big -t$T: /"
done
echo "vaf identical across -t (big): $(cmp -s $D/gpu_t1.vaf $D/gpu_t4.vaf && cmp -s $D/gpu_t1.vaf $D/gpu_t16.vaf && echo yes || echo NO)"

# host-only ingest (reader + block loop, no device): the ceilings of the CLI
python - "$D/big.fq" "$K" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc
fn, k = sys.argv[1], int(sys.argv[2])
st, _ = vafc.scan_file(fn, k)
print("host ingest only, one reader thread: %.0f Mbases/s" % (st.bases / st.seconds / 1e6))
for t in (4, 16):
    st2, _ = vafc.scan_file_parallel(fn, k, threads=t)
    assert (st2.bases, st2.seqs, st2.blocks) == (st.bases, st.seqs, st.blocks)
    print("host ingest only, parallel reader -t %d: %.0f Mbases/s" % (t, st2.bases / st2.seconds / 1e6))
PY

# gzip input (what sequencers deliver): zlib inflate bounds both programs
gzip -1 -c $D/r.fq > $D/r.fq.gz
timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -k $K -p $D/pat.txt -o $D/gpu_gz.vaf $D/r.fq.gz 2> $D/gpu_gz.err
grep -E "Speed" $D/gpu_gz.err | sed "s/^/gpu gz: /"
timeout -k 10 600 oracle/_ref/vaf-counter -v -t 1 -k $K -p $D/pat.txt -o $D/ref_gz.vaf $D/r.fq.gz 2> $D/ref_gz.err
grep -E "Speed" $D/ref_gz.err | sed "s/^/ref gz -t1: /"
echo "gz vaf identical: $(cmp -s $D/gpu_gz.vaf $D/ref_gz.vaf && echo yes || echo NO)"
