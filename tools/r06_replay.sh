#!/bin/bash
# Partitioned-mode rank replay at RMAT-26, N = 8 (tools/part_replay.py): bulk combine and
# 2^22-edge windows. Usage: bash tools/r06_replay.sh <tag>
set -o pipefail
TAG=${1:-r06c}
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/part_replay.py --ranks 8 --out $O/replay_bulk.json > $O/replay_bulk.log 2>&1 || { echo "bulk rc=$?"; tail -20 $O/replay_bulk.log; exit 1; }
grep -E "T1|digest_equal|efficiency|rank_ms_max|over_V" $O/replay_bulk.log
timeout -k 10 500 python -u tools/part_replay.py --ranks 8 --window-log 22 --out $O/replay_w22.json > $O/replay_w22.log 2>&1 || { echo "w22 rc=$?"; tail -20 $O/replay_w22.log; exit 1; }
grep -E "T1|digest_equal|efficiency|rank_ms_max|over_V" $O/replay_w22.log
