"""Kernel timeline of a rocprofv3 --kernel-trace database (rocpd sqlite): per kernel
name the dispatch count, summed and average duration, plus GPU busy time (union of
all dispatch intervals), idle gaps and the time with >= 2 kernels in flight.
python tools/timeline.py <run_results.db> [first_ns_offset_ms]"""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
src = "kernels" if "kernels" in views else [v for v in views if "kernel" in v.lower()][0]
cols = [r[1] for r in db.execute("pragma table_info(%s)" % src)]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = list(db.execute("select %s, start, end from %s order by start" % (name_col, src)))
if not rows:
    sys.exit("no kernels")
skip_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
t0 = rows[0][1] + skip_ms * 1e6
rows = [r for r in rows if r[1] >= t0]
agg = defaultdict(lambda: [0, 0.0])
for n, s, e in rows:
    k = n.split("(")[0].replace("void ", "")[:60]
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e3
for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-60s %7d %12.1f us %9.2f us avg" % (k, c, us, us / c))
ev = sorted([(s, 1) for _, s, _ in rows] + [(e, -1) for _, _, e in rows])
busy = multi = 0.0
depth = 0
last = ev[0][0]
for t, d in ev:
    if depth >= 1:
        busy += t - last
    if depth >= 2:
        multi += t - last
    depth += d
    last = t
span = ev[-1][0] - ev[0][0]
print("span %.1f us, busy %.1f us (%.1f%%), >=2 in flight %.1f us, idle %.1f us"
      % (span / 1e3, busy / 1e3, 100 * busy / span, multi / 1e3, (span - busy) / 1e3))
