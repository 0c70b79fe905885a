#!/bin/bash
# Round-5 first probe: young-table anatomy (configs 2 and 4), the config-2 bench line and the
# N = 8 rank replay's row statistics, product build (times) and debug build (counts).
set -o pipefail
O=gpurun_out/${1:-r05a}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 240 python tools/fold_stats.py r20 > $O/r20_times.txt 2>&1 &&
GS_LIB_VARIANT=debug timeout -k 10 240 python tools/fold_stats.py r20 --passes 1 > $O/r20_counts.txt 2>&1 &&
timeout -k 10 240 python tools/fold_stats.py bip > $O/bip_times.txt 2>&1 &&
GS_LIB_VARIANT=debug timeout -k 10 240 python tools/fold_stats.py bip --passes 1 > $O/bip_counts.txt 2>&1 &&
timeout -k 10 240 python bench.py --scale 20 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_r20.json 2> $O/bench_r20.err &&
timeout -k 10 300 python tools/rank_replay.py --row-stats --reps 1 --lag 2 > $O/replay_times.txt 2>&1 &&
GS_LIB_VARIANT=debug timeout -k 10 400 python tools/rank_replay.py --row-stats --reps 1 --lag 2 > $O/replay_counts.txt 2>&1
echo "rc=$?"
