#!/bin/bash
# One-rank exchange-path bench (RCCL, bench.py --exchange) on builds of earlier commits
# (git worktrees under bisect_x/, each built in-tree), to locate a step-time change.
# Usage (GPU box): tools/bisect_exch.sh <sha> ...   -> gpurun_out/bisect_exch_<sha>.log
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for c in "$@"; do
  cd $R/bisect_x/$c || exit 2
  timeout -k 10 200 python3 -u bench.py --exchange --steps 3 --warmup 1 --no-cpu-baseline --no-profile-pass > $R/gpurun_out/bisect_exch_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $R/gpurun_out/bisect_exch_$c.log)"
  [ $rc -eq 0 ] || { echo "stopping: rc $rc"; exit $rc; }
done
