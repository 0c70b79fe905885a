#!/bin/bash
# Round 5: rank 0 of the N = 8 RMAT-26 replay on the final build (VERDICT r4 item 1's evidence file): the replay
# (projected efficiency), then phase by phase with the debug build's fold counters.
set -o pipefail
O=gpurun_out/${1:-r05z}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python tools/rank_replay.py --reps 3 --lag 2 > $O/replay.txt 2>&1 || exit 1
timeout -k 10 300 python tools/rank_replay.py --row-stats --reps 1 --lag 2 > $O/replay_rows.txt 2>&1 || exit 1
GS_LIB_VARIANT=debug timeout -k 10 400 python tools/rank_replay.py --row-stats --reps 1 --lag 2 > $O/replay_counts.txt 2>&1
