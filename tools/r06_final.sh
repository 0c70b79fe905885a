#!/bin/bash
# Round 6 final-build evidence, third call (after tools/profile_round.sh <tag> and
# tools/final_round.sh <tag>): the one-rank partitioned line, per-dispatch traces of the config-2
# and config-4 steps, and the RMAT-26 N = 8 partitioned replays (bulk and 2^22-edge windows).
# Usage (repo root on the GPU box): bash tools/r06_final.sh <tag>
set -u
TAG=${1:-r06f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final_$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --exchange --combine partitioned --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_part1.out 2> $O/bench_part1.err || { echo "bench_part1 failed rc=$?"; exit 1; }
echo "bench_part1 ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/bip_$TAG -o run -- python3 $R/bench.py --workload bip --steps 3 --warmup 1 --profile-only --no-profile-pass > $O/bip_trace.log 2>&1 || { echo "bip trace failed rc=$?"; exit 1; }
python3 $R/tools/step_dispatches.py "$(find /tmp/bip_$TAG -name '*.db' | head -1)" 1.2 > $O/bip_dispatches.txt
rm -rf /tmp/bip_$TAG
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/r20_$TAG -o run -- python3 $R/bench.py --scale 20 --steps 3 --warmup 1 --profile-only --no-profile-pass --no-cpu-baseline > $O/r20_trace.log 2>&1 || { echo "r20 trace failed rc=$?"; exit 1; }
python3 $R/tools/step_dispatches.py "$(find /tmp/r20_$TAG -name '*.db' | head -1)" 0.8 > $O/r20_dispatches.txt
rm -rf /tmp/r20_$TAG
echo "traces ok"
cd $R
for M in 0 22; do
  timeout -k 10 500 python -u tools/part_replay.py --ranks 8 --window-log $M --out $O/replay_w$M.json > $O/replay_w$M.log 2>&1 \
    || { echo "replay w$M failed rc=$?"; tail -5 $O/replay_w$M.log; exit 1; }
  echo "replay w$M ok"
done
