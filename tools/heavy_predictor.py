"""CPU study (round 6): how well stage 0's stop state predicts a heavy
history's remaining lane-mode iterations, and the lane utilisation of
groups of 64 formed in list order, sorted by a predictor, or bucketed by it
(tools/heavy_emu.py runs each heavy history; HISTORY.md §10, round 6).

    python tools/heavy_predictor.py n_hist budget config
"""
import sys, os, numpy as np
sys.path[:0]=['tools','quickcheck-state-machine-distributed_amd','oracle']
import heavy_emu as he  # noqa: E402
from qsmd import gen
import oracle_c
n=int(sys.argv[1]); budget=int(sys.argv[2]); cfg=sys.argv[3]
hdr, ev, _ = gen.generate_config(cfg, 0, n, threads=8)
st_o, nd_o, _ = oracle_c.check_batch(2, hdr, ev, threads=8)
heavy = np.nonzero(nd_o > budget)[0]
rows=[]
for i in heavy:
    hd=hdr[i]; h=he.Hist(ev[int(hd["ev_off"]): int(hd["ev_off"]) + int(hd["n_ev"])])
    s, nd, it1, it0, desc, hits = he.run(h, budget, 32, 128)
    inf=he.run.info
    rem_ev = int(hd["n_ev"]) - 2*inf.get("depth",0)
    rows.append((it1, inf.get("depth",0), inf.get("cand",0), inf.get("stack_untried",0), inf.get("fails",0), rem_ev, int(hd["n_ev"])))
R=np.array(rows)
it=R[:,0]
def util(order):
    x=it[order]; g=len(x)//64; x=x[:g*64].reshape(g,64); return x.sum()/(x.max(1).sum()*64), x.max(1).sum()
print("heavy", len(it), "list order util %.3f sum %d" % util(np.arange(len(it))))
print("perfect sort util %.3f sum %d" % util(np.argsort(-it)))
names=["depth","cand","stack_untried","fails","rem_ev"]
for k,nm in enumerate(names):
    f=R[:,k+1]
    c=np.corrcoef(f,it)[0,1]
    # bucket into 8 quantile buckets, stable within bucket (list order)
    order=np.argsort(-f, kind="stable")
    print(nm, "corr %.3f" % c, "sorted-by util %.3f sum %d" % util(order))
su=R[:,3].astype(float); dp=R[:,1].astype(float); cd=R[:,2].astype(float)
for nm,f in [("su+cand",su+cd),("su+0.5dp",su+0.5*dp),("su*dp",su*(dp+1)),("su+dp",su+dp)]:
    print(nm, "corr %.3f" % np.corrcoef(f,it)[0,1], "util %.3f sum %d" % util(np.argsort(-f,kind="stable")))
# bucketed: 8 / 16 buckets by stack_untried value (clipped), list order within
for nb in (4,8,16):
    b=np.minimum(su.astype(int), nb-1)
    order=np.argsort(-b, kind="stable")
    print("buckets", nb, "util %.3f sum %d" % util(order), np.bincount(b.astype(int)))
