#!/usr/bin/env python3
"""Pass rate of the flank-bitmap prefilter (vafc_common.h vc_flank_mark) on the
benchmark panel, CPU only: the exact 2^20-bit set of every key's first and
last ten bases (both strands), queried with 4M uniform random k-mers.
    python tools/flank_fp.py
"""
import os, sys, tempfile
import numpy as np
ROOT=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, os.path.join(ROOT,"kmer-cnt_amd")); sys.path.insert(0, os.path.join(ROOT,"tools"))
import vafc, vafc_synth as S
def revcomp(x,K):
    r=np.zeros_like(x)
    for _ in range(K):
        r=(r<<np.uint64(2))|(np.uint64(3)-(x&np.uint64(3))); x=x>>np.uint64(2)
    return r
panel=S.make_panel(S.read_bed(S.default_bed_path()))
for K in (21,31,25,17):
    d=tempfile.mkdtemp(); pat=os.path.join(d,"p.txt"); panel.write_patterns(pat,K)
    keys,_,_=vafc.load_patterns(pat).keys(K)
    keys=np.unique(np.asarray(keys,dtype=np.uint64))
    allk=np.concatenate([keys,revcomp(keys,K)])
    M=np.uint64((1<<20)-1)
    last=allk&M; first=(allk>>np.uint64(2*K-20))&M
    bm=np.zeros(1<<20,bool); bm[last]=True; bm[first]=True
    dens=bm.mean()
    q=np.random.default_rng(1).integers(0,1<<(2*K),size=4_000_000,dtype=np.uint64)
    ql=q&M; qf=(q>>np.uint64(2*K-20))&M
    fp=(bm[ql]&bm[qf]).mean()
    print(K,"keys",len(keys),"distinct10",bm.sum(),"density %.4f"%dens,"FP %.4f%%"%(100*fp))
