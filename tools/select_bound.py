"""Bracket quality for a select-free threshold pipeline (VERDICT r05 "next" #2, design (a)).

    python tools/select_bound.py FRAMES hard|bench

For 8 pairs of the covers80-shaped corpus: the exact distance matrix D (oracle), the exact row and
column order statistics k0 = floor((n - 1) kappa), k0 + 1, and three ways to bracket them BEFORE
the lines are selected:
  * (row|col, S, eps): the exact thresholds of every S-th line, the bracket of a line between two
    sampled lines = [min, max] of their two order statistics, widened by eps relative;
  * (row|col, subS, z): the kappa-quantile of every S-th element of the line itself, +- z standard
    errors of a sample quantile.
Per strategy: the fraction of lines whose exact order statistics fall outside the bracket (a miss:
the line needs the full select anyway) and the number of line elements inside the bracket (the
candidates the walk would have to emit and a resolve pass would have to select among).
Output: profiles/r06/select_bound/brackets_<frames>.txt.
"""
import os, sys, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'acoss-1_amd')]
import oracle
from acoss import synthetic
frames=int(sys.argv[1]); kind=sys.argv[2]
if kind=='hard':
    tracks, labels = synthetic.make_hard_corpus("covers80", frames=frames, seed=20250101)
else:
    tracks, labels = synthetic.make_corpus("covers80", frames=frames, seed=20250101)
rng=np.random.default_rng(1)
pairs=[(0,1),(2,3)]+[tuple(sorted(rng.choice(len(tracks),2,replace=False))) for _ in range(6)]
kappa=0.095
def order_stats(D, axis):
    n=D.shape[axis]; q=(n-1)*kappa; k0=int(np.floor(q))
    s=np.sort(D,axis=axis)
    if axis==1: return s[:,k0], s[:,min(k0+1,n-1)], s
    return s[k0,:], s[min(k0+1,n-1),:], s
res={}
for (a,b) in pairs:
    r=oracle.crp_pair(tracks[a],tracks[b])
    D=oracle.crp_dist(tracks[a],tracks[b],k=r['oti']).astype(np.float64)
    for axis,name in ((1,'row'),(0,'col')):
        lo_t, hi_t, s = order_stats(D, axis)
        T = lo_t  # bracket centre proxy: exact k0-th of sampled lines
        nl=len(T); n=D.shape[axis]
        for stride in (4,8,16):
            for eps in (0.0,0.02,0.05):
                miss=0; cand=[]
                for i in range(nl):
                    a0=(i//stride)*stride; b0=min(a0+stride, nl-1)
                    lo=min(lo_t[a0],lo_t[b0],hi_t[a0],hi_t[b0])*(1-eps); hi=max(lo_t[a0],lo_t[b0],hi_t[a0],hi_t[b0])*(1+eps)
                    line = D[i] if axis==1 else D[:,i]
                    if not (lo<=lo_t[i] and hi_t[i]<=hi): miss+=1
                    cand.append(np.sum((line>=lo)&(line<=hi)))
                res.setdefault((name,stride,eps),[]).append((miss/nl, np.mean(cand), np.percentile(cand,99)))
        # subsample quantile estimate
        for sub in (4,8):
            for z in (3,4):
                miss=0;cand=[]
                for i in range(nl):
                    line = D[i] if axis==1 else D[:,i]
                    smp=np.sort(line[::sub]); ns=len(smp)
                    sd=np.sqrt(kappa*(1-kappa)/ns)
                    ql=max(0,int(np.floor((kappa-z*sd)*(ns-1)))); qh=min(ns-1,int(np.ceil((kappa+z*sd)*(ns-1)))+1)
                    lo=smp[ql]; hi=smp[qh]
                    if not (lo<=lo_t[i] and hi_t[i]<=hi): miss+=1
                    cand.append(np.sum((line>=lo)&(line<=hi)))
                res.setdefault((name,'sub%d'%sub,z),[]).append((miss/nl,np.mean(cand),np.percentile(cand,99)))
for k,v in res.items():
    v=np.array(v); print(k, "miss %.4f  cand mean %.1f  p99 %.1f"%(v[:,0].mean(), v[:,1].mean(), v[:,2].max()))
