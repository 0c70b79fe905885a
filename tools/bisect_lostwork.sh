#!/bin/bash
# Re-run round 2's lost-work reproduction (8 emulated ranks, 32 HW queues, highest-
# priority comm streams) on builds of earlier commits (git worktrees under bisect/,
# each patched back to highest-priority comm streams and built in-tree).
# Usage (GPU box): tools/bisect_lostwork.sh <sha> ...   -> gpurun_out/bisect_<sha>.log
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for c in "$@"; do
  cd $R/bisect/$c || exit 2
  GPU_MAX_HW_QUEUES=32 timeout -k 10 200 python3 -u tools/emu_check.py --ranks 8 --passes 3 > $R/gpurun_out/bisect_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc $(tail -1 $R/gpurun_out/bisect_$c.log)"
  case $rc in 0|1) ;; *) echo "stopping: rc $rc"; exit $rc;; esac
done
