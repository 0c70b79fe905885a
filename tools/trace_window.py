"""Print the kernels of a rocprofv3 --kernel-trace database (rocpd sqlite) that start
inside a time window, one line each: start/end relative to the window (us), duration,
queue / stream id when the schema has one, short name. The window starts
<offset_ms> after the first kernel whose name contains <anchor> (default k_fold).
Used to read the schedule of the exchange loop (which stream waits for what).
python tools/trace_window.py <db> <offset_ms> <width_us> [anchor]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
src = "kernels" if "kernels" in views else [v for v in views if "kernel" in v.lower()][0]
cols = [r[1] for r in db.execute("pragma table_info(%s)" % src)]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
extra = [c for c in ("queue_id", "stream_id") if c in cols]
q = "select %s, start, end%s from %s order by start" % (name_col, "".join(", " + c for c in extra), src)
rows = list(db.execute(q))
anchor = sys.argv[4] if len(sys.argv) > 4 else "k_fold"
first = next(r[1] for r in rows if anchor in r[0])
t0 = first + float(sys.argv[2]) * 1e6
t1 = t0 + float(sys.argv[3]) * 1e3
for r in rows:
    if t0 <= r[1] <= t1:
        nm = r[0].split("(")[0].replace("void ", "").split("::")[-1][:48]
        print("%9.2f %9.2f %8.2f %s %s" % ((r[1] - t0) / 1e3, (r[2] - t0) / 1e3, (r[2] - r[1]) / 1e3,
                                         " ".join(str(x) for x in r[3:]), nm))
