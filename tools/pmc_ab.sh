#!/bin/bash
# A/B of k_fold read requests and L2 hits under an environment setting:
# bash tools/pmc_ab.sh <tag> VAR=value ...  (one bench step, default settings)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
for kv in "$@"; do export "$kv"; done
OUT=$R/gpurun_out/pmcab_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/a -o run -- python3 $R/bench.py $ARGS > $OUT/a.log 2>&1 || exit 1
python3 - "$OUT/a" <<'PY'
import glob, sqlite3, sys
from collections import defaultdict
db = sqlite3.connect(glob.glob(sys.argv[1] + "/*.db")[0])
agg = defaultdict(lambda: defaultdict(list))
for k, c, v in db.execute("select kernel_name, counter_name, value from counters_collection"):
    if "k_fold" in k:
        agg[k.split("(")[0]][c].append(v)
for k, cs in agg.items():
    n = len(cs["TCC_EA0_RDREQ_sum"])
    tail = lambda c: sorted(cs[c])[n // 2]  # median launch
    h, m = tail("TCC_HIT_sum"), tail("TCC_MISS_sum")
    print("%s launches %d median RDREQ/launch %.0f (%.3f per 2^20-edge) L2 hit %.3f" % (k, n, tail("TCC_EA0_RDREQ_sum"), tail("TCC_EA0_RDREQ_sum") / 2**20, h / (h + m)))
PY
