#!/bin/bash
# Kernel trace of the ingest step, single pass (fused) and two-pass, on the GPU box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ingest_ktrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${MODES:-1 0}; do
  GS_PARSE_MODE=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/ik_$v -o run -- python3 $R/bench.py --workload ingest --steps 5 --warmup 1 --profile-only > $O/log_$v.txt 2>&1 || { echo "trace $v failed"; exit 1; }
  DB=$(find /tmp/ik_$v -name "*.db" | head -1)
  python3 $R/tools/timeline.py "$DB" 0 > $O/timeline_mode$v.txt
  echo "== mode=$v"; head -8 $O/timeline_mode$v.txt
  rm -rf /tmp/ik_$v
done
