"""Per-dispatch listing of the last step of a rocprofv3 --kernel-trace database (rocpd
sqlite): every kernel dispatch in the final `window_ms` of the trace, with its start
relative to the first of them, duration, idle gap since the previous dispatch ended
(GPU-wide) and its queue / stream when the trace has them. Used to see where a step's
time goes between kernels (the config-4 step).
python tools/step_dispatches.py <run_results.db> <window_ms> [name filter ...]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
window_ms = float(sys.argv[2])
filt = sys.argv[3:]
views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
src = "kernels" if "kernels" in views else [v for v in views if "kernel" in v.lower()][0]
cols = [r[1] for r in db.execute("pragma table_info(%s)" % src)]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
extra = [c for c in ("queue_id", "stream_id", "queue", "stream") if c in cols]
q = "select %s, start, end%s from %s order by start" % (name_col, "".join(", " + c for c in extra), src)
rows = list(db.execute(q))
if not rows:
    sys.exit("no kernels")
t_end = max(r[2] for r in rows)
rows = [r for r in rows if r[1] >= t_end - window_ms * 1e6]
if filt:
    rows = [r for r in rows if any(f in r[0] for f in filt)]
print("# columns: %s; %d dispatches in the last %.3f ms" % (", ".join(cols), len(rows), window_ms))
t0 = rows[0][1]
last_end = rows[0][1]
busy_end = rows[0][1]
print("%10s %9s %9s  %-44s %s" % ("start_us", "dur_us", "gap_us", "kernel", " ".join(extra)))
for r in rows:
    n, s, e = r[0], r[1], r[2]
    gap = max(0, s - busy_end)
    busy_end = max(busy_end, e)
    k = n.split("(")[0].replace("void ", "")
    k = k[k.find("gs::") + 4:] if "gs::" in k else k
    print("%10.1f %9.2f %9.2f  %-44s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, k[:44],
                                             " ".join(str(x) for x in r[3:])))
print("# span %.1f us, GPU busy until %.1f us" % ((rows[-1][2] - t0) / 1e3, (busy_end - t0) / 1e3))
