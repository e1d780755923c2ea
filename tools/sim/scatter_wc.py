#!/usr/bin/env python3
"""Round 5: host model of scatter write-combining -- with the nslots hottest (workgroup, tile)
runs given an L-line LDS ring, how many store transactions per record remain?  (DESIGN.md
§18; the device diagnostic confirmed ~65 % of the records parked, 3.9 per flushed line.)"""
import numpy as np, sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', 'astro-sph-tools_amd'))
from asp_amd.plummer import plummer
p = plummer(4_000_000, seed=1, h_law="pixel", grid=4096)
x,y = p["pos"][:,0], p["pos"][:,1]
G=4096; ext=4.0; ps=2*ext/G
ix = np.floor((x+ext)/ps).astype(np.int64); iy=np.floor((y+ext)/ps).astype(np.int64)
ok=(ix>=0)&(ix<G)&(iy>=0)&(iy<G)
t = (ix[ok]//64)*64 + iy[ok]//64
cnt = np.bincount(t, minlength=4096).astype(float)
pt = cnt/cnt.sum(); frac_in = ok.mean()
srt = np.sort(pt)[::-1]
for k in (128,256,384,512,768,1024,2048):
    print(k, "top tiles share", srt[:k].sum())
# per workgroup: 381 batches of 1024 particles
rng=np.random.default_rng(0)
nb=381; B=1024*frac_in
lam = pt*B
for NS, L in ((384,2),(512,2),(768,1),(768,2),(1024,1),(1536,1)):
    hot = np.argsort(pt)[::-1][:NS]
    tot=0; trans=0
    for t in hot:
        k = rng.poisson(lam[t], nb)
        # ring of L lines of 4 records; pending start line = cursor//4
        cur=0; 
        for kk in k:
            s0=cur; s1=cur+kk
            Ls = s0//4
            # records with line < Ls+L go to LDS, others bypass
            lim = (Ls+L)*4
            inl = max(0, min(s1,lim)-s0); by = kk-inl
            trans += by
            # complete lines flushed: lines fully claimed with end <= s1 among lines [Ls, Ls+L)
            endc = min(s1, lim)
            trans += max(0, endc//4 - Ls)
            cur=s1
        trans += 1 if cur%4 else 0
        tot += k.sum()
    cold = B*nb - tot
    print(NS, L, "LDS KB", NS*L*128/1024, "trans/record", (trans+cold)/(B*nb), "hot share", tot/(B*nb))
