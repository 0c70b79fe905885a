#!/bin/bash
# Kernel trace of rank 0's own folds, untracked vs tracked + takes (tools/rank_replay.py --own-only, N = 8 shard):
# where the tracking tax goes, per kernel.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/track_tax
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/tt -o run -- python3 $R/tools/rank_replay.py --ranks 8 --lag 2 --reps 3 --own-only > $O/log.txt 2>&1 || { tail -5 $O/log.txt; exit 1; }
cat $O/log.txt | grep "rank 0"
DB=$(find /tmp/tt -name "*.db" | head -1)
python3 $R/tools/timeline.py "$DB" 0 > $O/timeline.txt
head -14 $O/timeline.txt
