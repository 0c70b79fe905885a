"""Idle time between a group's own folds in rocprofv3 kernel traces (diagnostic): for each
trace directory under gpurun_out/, the gaps during which no tracked k_fold runs (gaps
longer than 3 ms -- between passes -- are left out).

    rocprofv3 --kernel-trace -d gpurun_out/<dir> -o run -- python3 bench.py --exchange ...
    python3 tools/fold_gaps.py <dir> [<dir> ...]
"""
import glob
import sqlite3
import sys

import numpy as np

for d in sys.argv[1:]:
    f = glob.glob("gpurun_out/%s/**/*.db" % d, recursive=True)[0]
    db = sqlite3.connect(f)
    rows = list(db.execute("select name, start, end from kernels order by start"))
    folds = [r for r in rows if "k_fold<false, true" in r[0]]
    iv = sorted((r[1], r[2]) for r in folds)
    gaps, ce = [], iv[0][1]
    for a, b in iv[1:]:
        if a > ce:
            if a - ce < 3e6:
                gaps.append((a - ce) / 1e3)
            ce = b
        else:
            ce = max(ce, b)
    g = np.array(gaps)
    print("%s folds %d, gaps %d, total %.2f ms, p50 %.1f us, p90 %.1f" %
          (d, len(folds), len(g), g.sum() / 1e3, np.median(g), np.percentile(g, 90)))
