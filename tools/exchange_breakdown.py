"""Per-phase GPU time of the N-rank exchange, from a rocprofv3 kernel trace of
tools/emulated_scaling.py (all ranks on one GPU, so GPU busy time = the sum of
every rank's work).

    rocprofv3 --kernel-trace -d D -o run -- python3 tools/emulated_scaling.py --ranks N --reps 1
    python3 tools/exchange_breakdown.py D --ranks N --passes 2

Phases (kernel, how it is told apart):
  own fold     k_fold launches over one 2^micro-edge micro-batch (grid = 2^micro / 256)
  remote fold  every other k_fold launch (the gathered rows of the other ranks)
  stage        k_stage (delta list -> contiguous rows)
  copies       the emulated all-gather (device copy kernels / copy engine)
  other        headers, reports, resets, ...
The trace covers the plain 1-rank pass too: its folds are the launches before the
first k_stage, reported separately as the baseline.
"""
import argparse
import glob
import json
import os
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--ranks", type=int, required=True)
    ap.add_argument("--passes", type=int, default=2, help="timed passes per phase in the trace (reps + 1)")
    ap.add_argument("--micro", type=int, default=20)
    a = ap.parse_args()
    n, micro = a.ranks, a.micro
    dbs = glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True)
    db = sqlite3.connect(dbs[0])
    views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
    src = "kernels" if "kernels" in views else [v for v in views if "kernel" in v.lower()][0]
    cols = [r[1] for r in db.execute("pragma table_info(%s)" % src)]
    gx = [c for c in cols if "grid" in c.lower() and c.lower().endswith("x")]
    wx = [c for c in cols if "workgroup" in c.lower() and c.lower().endswith("x")]
    rows = list(db.execute("select name, start, end, %s, %s from %s order by start" % (gx[0], wx[0], src)))
    first_stage = next((s for nm, s, e, g, w in rows if "k_stage" in nm), None)
    acc = {}
    spans = {}  # phase -> kernel intervals, for its busy time (union)
    own_grid = {1 << micro, (1 << micro) // 256}  # threads or workgroups, whichever the trace records

    def add(k, dt):
        a = acc.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += dt
        spans.setdefault(k, []).append(cur)

    for nm, s, e, g, w in rows:
        dt = (e - s) / 1e6
        cur = (s, e)
        if first_stage is not None and s < first_stage:
            add("plain fold (1 rank, no exchange)" if "k_fold" in nm else "plain other", dt)
            continue
        if "k_fold" in nm:
            add("own fold" if g in own_grid else "remote fold", dt)
        elif "k_stage" in nm:
            add("stage", dt)
        elif "copy" in nm.lower() or "Copy" in nm:
            add("copies", dt)
        else:
            add("other", dt)
    for t in ("memory_copies", "memory_copy"):
        if t in views:
            ms = sum((e - s) / 1e6 for s, e in db.execute("select start, end from %s" % t))
            cnt = db.execute("select count(*) from %s" % t).fetchone()[0]
            acc["copy engine"] = [cnt, ms]
            break
    def union_ms(iv):
        busy, cs, ce = 0, None, None
        for s_, e_ in sorted(iv):
            if ce is None or s_ > ce:
                if ce is not None:
                    busy += ce - cs
                cs, ce = s_, e_
            else:
                ce = max(ce, e_)
        return (busy + (ce - cs if ce is not None else 0)) / 1e6

    group = [iv for k, v in spans.items() if not k.startswith("plain") for iv in v]
    out = {"ranks": n,
           "busy_ms_per_pass": {k: round(union_ms(v) / a.passes, 2) for k, v in spans.items()},
           "group_busy_ms_per_pass": round(union_ms(group) / a.passes, 2),
           "group_wall_ms_per_pass": round((max(e for _, e in group) - min(s for s, _ in group)) / 1e6 / a.passes, 2)
           if group else 0.0, "kernel_ms_per_pass": {k: round(v[1] / a.passes, 2) for k, v in acc.items()},
           "launches_per_pass": {k: v[0] // a.passes for k, v in acc.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
