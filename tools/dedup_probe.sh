#!/bin/bash
# Build and profile tools/dedup_probe.hip: timings + TCC_EA0_RDREQ per edge of the
# dedup stage's two passes. Output under gpurun_out/dedup/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/dedup
mkdir -p $OUT
BIN=$R/tools/bin/dedup_probe
cd /tmp && export TMPDIR=/tmp
for L in 22 23; do
  timeout -k 10 120 $BIN $L 64 > $OUT/t$L.json
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/p$L -o run -- $BIN $L 64 > $OUT/p$L.log 2>&1
  python3 - "$OUT/p$L" "$L" <<'PY'
import glob, sqlite3, sys
from collections import defaultdict
db = sqlite3.connect(glob.glob(sys.argv[1] + "/*.db")[0])
agg = defaultdict(lambda: defaultdict(list))
for k, c, v in db.execute("select kernel_name, counter_name, value from counters_collection"):
    if "k_dd" in k:
        agg[k.split("(")[0]][c].append(v)
for k, cs in agg.items():
    n = len(cs["TCC_EA0_RDREQ_sum"])
    med = lambda c: sorted(cs[c])[n // 2]
    h, m = med("TCC_HIT_sum"), med("TCC_MISS_sum")
    print("table 2^%s %s launches %d RDREQ/edge %.3f L2 hit %.3f" % (sys.argv[2], k, n, med("TCC_EA0_RDREQ_sum") / 2**20, h / (h + m)))
PY
done
cat $OUT/t*.json
