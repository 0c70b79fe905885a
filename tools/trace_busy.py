"""Busy/idle split of a rocprofv3 kernel trace (diagnostic): per kernel name, the
launches, summed duration and the union of its intervals; then the union over all
kernels and the wall span, within the LAST `--window-ms` of the trace (the timed
step of a bench run).

    python tools/trace_busy.py <rocprofv3 -d dir> [--window-ms 60]
"""
import argparse
import glob
import json
import os
import sqlite3


def union_ns(iv):
    busy, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return busy + (ce - cs if ce is not None else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--window-ms", type=float, default=60.0)
    a = ap.parse_args()
    db = sqlite3.connect(glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)[0])
    views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
    src = "kernels" if "kernels" in views else [v for v in views if "kernel" in v.lower()][0]
    rows = list(db.execute("select name, start, end from %s" % src))
    end = max(e for _, _, e in rows)
    lo = end - a.window_ms * 1e6
    rows = [(n.split("(")[0].split("::")[-1], s, e) for n, s, e in rows if s >= lo]
    per = {}
    for n, s, e in rows:
        per.setdefault(n, []).append((s, e))
    out = {"window_ms": a.window_ms,
           "span_ms": round((max(e for _, _, e in rows) - min(s for _, s, _ in rows)) / 1e6, 3),
           "busy_ms": round(union_ns([(s, e) for _, s, e in rows]) / 1e6, 3),
           "kernels": {n: {"launches": len(v), "sum_ms": round(sum(e - s for s, e in v) / 1e6, 3),
                           "busy_ms": round(union_ns(v) / 1e6, 3)} for n, v in sorted(per.items())}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
