"""Idle periods of the GPU in the last `window_ms` of a rocprofv3 --kernel-trace database: the
intervals covered by no kernel on any stream, largest first, with the kernels that end before and
start after each. usage: python tools/gaps.py <results.db> [window_ms] [top]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    window = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    c = sqlite3.connect(db)
    rows = list(c.execute("select start, end, name, stream_id from kernels order by start"))
    t_end = max(r[1] for r in rows)
    t0 = t_end - window * 1e6
    rows = [r for r in rows if r[1] > t0]
    gaps, busy_end, last = [], t0, None
    for s, e, name, st in rows:
        if s > busy_end and last is not None:
            gaps.append((s - busy_end, busy_end, last, (name, st)))
        if e > busy_end:
            busy_end, last = e, (name, st)
    idle = sum(g[0] for g in gaps)
    print("window %.1f ms: %d kernels, idle %.3f ms in %d gaps" % (window, len(rows), idle / 1e6, len(gaps)))
    for d, at, before, after in sorted(gaps, reverse=True)[:top]:
        print("%9.1f us at -%8.3f ms  after %-40s [%s]  before %-40s [%s]" % (
            d / 1e3, (t_end - at) / 1e6, before[0][:40], before[1], after[0][:40], after[1]))


if __name__ == "__main__":
    main()
