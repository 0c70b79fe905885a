"""Per-window anatomy of the config-5 loop (diagnostic): from a rocprofv3
--kernel-trace --hip-runtime-trace database of host/bin/window_latency, the fold
kernel's duration, the idle gap between consecutive windows' kernels, the HIP calls
issued per window, and one window's timeline.
    rocprofv3 --kernel-trace --hip-runtime-trace -d out -o run -- host/bin/window_latency 22 16 6
    python tools/window_anatomy.py out/run_results.db
"""
import sqlite3,numpy as np,sys,collections
c=sqlite3.connect(sys.argv[1])
views=[r[0] for r in c.execute("select name from sqlite_master where type='view'")]
k=c.execute("select name,start,end from kernels order by start").fetchall()
fold=[(s,e) for n,s,e in k if 'k_fold' in n]
print("folds",len(fold))
# hip api
rs=c.execute("select name,start,end from regions order by start").fetchall()
cnt=collections.Counter(n for n,s,e in rs)
print(cnt.most_common(20))
# take last 500 folds; for each, list api calls between previous fold end and this fold end
fold=fold[-500:]
per=collections.defaultdict(list)
gaps=[];durs=[]
ri=0
import bisect
starts=[s for n,s,e in rs]
for j in range(1,len(fold)):
    a=fold[j-1][1]; b=fold[j][1]
    durs.append((fold[j][1]-fold[j][0])/1e3); gaps.append((fold[j][0]-fold[j-1][1])/1e3)
    i0=bisect.bisect_left(starts,fold[j-1][0]); i1=bisect.bisect_left(starts,fold[j][0])
    for n,s,e in rs[i0:i1]: per[n].append((e-s)/1e3)
print("kernel p50 %.2f  gap p50 %.2f  period p50 %.2f"%(np.median(durs),np.median(gaps),np.median(np.diff([s for s,e in fold]))/1e3))
for n,v in per.items(): print("%-40s calls/window %.2f  p50 %.2f us"%(n,len(v)/(len(fold)-1),np.median(v)))
# timeline of one window
j=len(fold)-2
a=fold[j][0]; b=fold[j+1][1]
ev=[("K "+n[:30],s,e) for n,s,e in k if a<=s<=b]+[("A "+n,s,e) for n,s,e in rs if a<=s<=b]
ev.sort(key=lambda x:x[1])
for n,s,e in ev: print("%8.2f %8.2f %s"%((s-a)/1e3,(e-a)/1e3,n))
