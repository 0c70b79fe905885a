import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, gsamd as gs, oracle
s, d = oracle.rmat_edges(0x5EED0016, 14, 0, 1 << 16, True)
W = 1 << 13
before = {}
x = gs.Summary("cc", capacity_hint=1 << 14)
x.set_change_tracking(True)
for lo in range(0, len(s), W):
    hi = min(len(s), lo + W)
    x.fold(s[lo:hi], d[lo:hi])
    v, lab = x.take_changes()
    ov, ol = oracle.cc_labels(s[:hi], d[:hi])
    after = dict(zip(ov.tolist(), ol.tolist()))
    rows = dict(zip(v.tolist(), lab.tolist()))
    changed = {k for k, l in after.items() if before.get(k) != l}
    extra = set(rows) - changed
    missing = changed - set(rows)
    c = x.counters()
    print("window", lo // W, "rows", len(rows), "changed", len(changed), "extra", len(extra), "missing", len(missing),
          "ovf", c["ovf"], "nv", x.num_vertices(), "cap", x.table_capacity(), "capstats", x.capacity_stats())
    if extra:
        labs = {}
        for k in list(extra)[:5]:
            print("   extra", k, "label", rows[k], "before", before.get(k))
        from collections import Counter
        print("   extra labels", Counter(rows[k] for k in extra).most_common(5))
    before = after
