#!/bin/bash
# SQ stall counters of k_parse (text ingest), one rocprofv3 --pmc pass per group, on the
# GPU box from the repo root: where do k_parse's waves wait?
# Usage: bash tools/ingest_stalls.sh <tag> [bench args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stalls_$TAG
mkdir -p $OUT
ARGS="--workload ingest --steps 2 --warmup 0 --profile-only $*"
cd /tmp && export TMPDIR=/tmp
PASSES=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"
        "GRBM_GUI_ACTIVE GRBM_COUNT")
for P in "${PASSES[@]}"; do
  N=$(echo $P | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc_$N -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_$N.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $P failed rc=$rc"; tail -3 $OUT/pmc_$N.log; case $rc in 137|124|134|139) exit $rc;; esac; else echo "pmc $N ok"; fi
done
python3 - "$OUT" <<'PY'
import glob, os, sqlite3, sys
from collections import defaultdict
out = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for db in glob.glob(os.path.join(out, "pmc_*", "**", "*.db"), recursive=True):
    c = sqlite3.connect(db)
    for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        k = k.split("(")[0].replace("void ", "").split("::")[-1]
        agg[k][n].append(v)
with open(os.path.join(out, "summary.txt"), "w") as f:
    for k in sorted(agg):
        if "parse" not in k and "count_lines" not in k:
            continue
        line = "%s: " % k + ", ".join("%s=%.4g" % (n, sum(v) / len(v)) for n, v in sorted(agg[k].items()))
        print(line)
        f.write(line + "\n")
PY
rm -rf $OUT/pmc_*/
