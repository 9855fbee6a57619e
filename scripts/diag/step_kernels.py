"""Per-step time of the small memory-bound kernels (LN fwd/bwd, split-K reduce, column-sum
finalize) from a rocprofv3 rocpd database -- round 4 N>1-path slowdown probes."""
import sqlite3,collections,sys
db=sqlite3.connect(sys.argv[1])
rows=list(db.execute("select name,stream_id,queue_id,start,end from kernels order by start"))
st=[r[3] for r in rows if 'emb_ln_fwd' in r[0]]
print('steps ms',[round((b-a)/1e6,2) for a,b in zip(st,st[1:])])
for i,(a,b) in enumerate(zip(st,st[1:])):
    d=collections.defaultdict(float)
    for r in rows:
        if a<=r[3]<b:
            n=r[0]
            k='lnf' if 'ln_fwd_wave' in n else 'lnb' if 'ln_bwd_wave' in n else 'splitk' if 'splitk' in n else 'colsum' if 'colsum_fin' in n else None
            if k: d[k]+=(r[4]-r[3])/1e6
    print(i, {k:round(v,2) for k,v in d.items()})
