#!/bin/bash
# Where the drop-in CLI loses on gzip input (tools only): the CLI at several
# -t against the host-only ingest (inflate + kseq parse + block loop, no
# device) with the CLI's own chunk sizing and with 4 MiB chunks.
#   tools/gz_probe.sh [n_reads]
set -e
N=${1:-4000000}
D=${TMPDIR:-/tmp}/vafc_gz_probe; mkdir -p $D
trap "rm -rf $D" EXIT
python - "$D" "$N" <<'PY'
import sys; sys.path.insert(0, 'kmer-cnt_amd')
import vafc_synth as S
d, n = sys.argv[1], int(sys.argv[2])
p = S.grch38_panel(); p.write_patterns(d + '/pat.txt', 21)
S.write_fastq(d + '/r.fq', p, n, f_snp=0.01)
PY
gzip -1 -c $D/r.fq > $D/r1.fq.gz
cat $D/r1.fq.gz > /dev/null
for T in 8 12 16 24; do
  timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -t $T -k 21 -p $D/pat.txt -o $D/g_t$T.vaf $D/r1.fq.gz 2> $D/g_t$T.err
  grep -E "Speed" $D/g_t$T.err | sed "s/^/cli -t$T: /"
done
VAFC_GZ_PROFILE=1 timeout -k 10 300 kmer-cnt_amd/lib/vaf-counter -v -t 16 -k 21 -p $D/pat.txt -o $D/g_p.vaf $D/r1.fq.gz 2>&1 | grep -E "gzp|Speed" | sed "s/^/cli -t16 profiled: /"
python - "$D/r1.fq.gz" <<'PY'
import sys, time; sys.path.insert(0, 'kmer-cnt_amd')
import vafc
fn = sys.argv[1]
for t in (16,):
    for pb in (0, 4 << 20):
        st, _ = vafc.scan_file_parallel(fn, 21, threads=t, piece_bytes=pb)
        print("host-only ingest, %d workers, chunk %s: %.0f Mbases/s" % (t, pb or "adaptive", st.bases / st.seconds / 1e6))
    import numpy as np
    st = np.zeros(6, np.uint64)
    t0 = time.time(); n = vafc.lib().vc_gz_inflate_parallel(fn.encode(), t, 0, None, 0, st.ctypes.data); dt = time.time() - t0
    print("inflate only (counting the output), %d workers: %.0f MB/s of FASTQ text = %.0f Mbases/s" % (t, n / dt / 1e6, n / dt / 1e6 * 150 / 311))
PY
