"""Per-API host time from a rocprofv3 --hip-trace database:
python tools/hip_api_summary.py <run_results.db> [top]"""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
src = "regions" if "regions" in views else None
cols = [r[1] for r in db.execute("pragma table_info(%s)" % src)]
agg = defaultdict(lambda: [0, 0.0])
for name, s, e in db.execute("select name, start, end from %s" % src):
    a = agg[name]
    a[0] += 1
    a[1] += (e - s) / 1e3
for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print("%-40s %8d calls %10.1f us total %8.2f us avg" % (name[:40], n, us, us / n))
