"""Idle time between kernel dispatches of the training steps in a rocprofv3 (rocpd)
kernel trace, attributed to the (previous kernel -> next kernel) transition: where the
chip waits on launches, host work or cross-stream dependencies.

    python bench/prof_gaps.py gpurun_out/prof/run_results.db
"""
import sqlite3, collections, sys
db=sys.argv[1]
c=sqlite3.connect(db)
ks=c.execute("select name,start,end,stream_id from kernels order by start").fetchall()
marks=[i for i,k in enumerate(ks) if 'synth_images_kernel' in k[0]]
tot=collections.Counter(); num=collections.Counter()
for si in range(-6,-1):
    seg=ks[marks[si]:marks[si+1]]
    ev=sorted(seg,key=lambda k:k[1])
    end=ev[0][2]; prevn=ev[0][0]
    for n,s,e,q in ev[1:]:
        g=s-end
        if g>0:
            key=(prevn.split('(')[0].replace('void pmd::','')[:40], n.split('(')[0].replace('void pmd::','')[:40])
            tot[key]+=g; num[key]+=1
        if e>end: end=e; prevn=n
print("total idle per step %.1f us"%(sum(tot.values())/5e3))
for k,v in tot.most_common(15):
    print("%8.1f us/step %4d  %s -> %s"%(v/5e3, num[k]//5, k[0], k[1]))
