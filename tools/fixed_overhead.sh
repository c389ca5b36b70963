set -e
D=/tmp/vafc_fixed; mkdir -p $D
python - $D <<'PY'
import sys; sys.path.insert(0,'kmer-cnt_amd')
import vafc_synth as S
d=sys.argv[1]; p=S.grch38_panel(); p.write_patterns(d+'/pat.txt',21); S.write_fastq(d+'/r.fq',p,1000,f_snp=0.01)
PY
gzip -1 -c $D/r.fq > $D/r.fq.gz
for f in r.fq r.fq.gz; do for t in 4 16; do
  timeout -k 10 120 kmer-cnt_amd/lib/vaf-counter -v -t $t -k 21 -p $D/pat.txt -o $D/o.vaf $D/$f 2>&1 | grep -iE "time|Speed" | sed "s/^/$f -t$t: /"
done; done
