#!/bin/bash
# Quick end-to-end parity check on the GPU box: synthetic inputs, the HIP
# vaf-counter vs the reference binary built from /root/reference (oracle/_ref).
set -e
trap "rm -f gpurun_out/qc/*.fq" EXIT
D=gpurun_out/qc; mkdir -p $D
python - <<'PY'
import sys; sys.path.insert(0,'kmer-cnt_amd')
import vafc_synth as S
p=S.grch38_panel(); p.write_patterns('gpurun_out/qc/pat21.txt',21); p.write_patterns('gpurun_out/qc/pat31.txt',31)
S.write_fastq('gpurun_out/qc/r10k.fq',p,10000,f_snp=1.0)
S.write_fastq('gpurun_out/qc/r1m.fq',p,1000000,f_snp=0.05)
S.write_fastq('gpurun_out/qc/r1m_2.fq',p,1000000,seed=43,f_snp=0.05)
PY
for K in 21 31; do
  for F in r10k.fq "r1m.fq r1m_2.fq"; do
    tag=k${K}_$(echo $F | tr ' .' '__')
    (cd $D && timeout -k 10 300 ../../kmer-cnt_amd/lib/vaf-counter -v -k $K -p pat$K.txt -o gpu_$tag.vaf $F) 2> $D/gpu_$tag.err
    (cd $D && timeout -k 10 300 ../../oracle/_ref/vaf-counter -v -t 1 -k $K -p pat$K.txt -o ref_$tag.vaf $F) 2> $D/ref_$tag.err
    echo "$tag $(md5sum < $D/gpu_$tag.vaf) $(md5sum < $D/ref_$tag.vaf)"
    grep -E 'K-mers extracted|Speed' $D/gpu_$tag.err $D/ref_$tag.err
  done
done
