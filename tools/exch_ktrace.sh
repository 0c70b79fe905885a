#!/bin/bash
# Kernel trace of the one-rank RCCL exchange step vs the plain pass (per-kernel totals), on the GPU box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exch_ktrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in exch plain; do
  A="--steps 1 --warmup 1 --profile-only --no-cpu-baseline --no-profile-pass"
  [ $v = exch ] && A="$A --exchange"
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/xk_$v -o run -- python3 $R/bench.py $A > $O/log_$v.txt 2>&1 || { echo "trace $v failed"; tail -5 $O/log_$v.txt; exit 1; }
  DB=$(find /tmp/xk_$v -name "*.db" | head -1)
  python3 $R/tools/timeline.py "$DB" 0 > $O/timeline_$v.txt
  echo "== $v"; head -14 $O/timeline_$v.txt
  rm -rf /tmp/xk_$v
done
