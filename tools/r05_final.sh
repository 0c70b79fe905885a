#!/bin/bash
# Round 5 final-build evidence, second call: the GPU suite, smoke, every bench line (tools/final_round.sh) and
# per-dispatch traces of the config-4 and config-2 steps. Run after tools/profile_round.sh <tag> (first call), whose
# traffic files the bench lines read by library hash.
# Usage (repo root on the GPU box): bash tools/r05_final.sh <tag>
set -u
TAG=${1:-r05f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/final_round.sh $TAG || exit 1
O=$R/gpurun_out/final_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/bip_$TAG -o run -- python3 $R/bench.py --workload bip --steps 3 --warmup 1 --profile-only --no-profile-pass > $O/bip_trace.log 2>&1 || { echo "bip trace failed rc=$?"; exit 1; }
DB=$(find /tmp/bip_$TAG -name "*.db" | head -1)
python3 $R/tools/step_dispatches.py "$DB" 1.2 > $O/bip_dispatches.txt
rm -rf /tmp/bip_$TAG
echo "bip trace ok"
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/r20_$TAG -o run -- python3 $R/bench.py --scale 20 --steps 3 --warmup 1 --profile-only --no-profile-pass --no-cpu-baseline > $O/r20_trace.log 2>&1 || { echo "r20 trace failed rc=$?"; exit 1; }
DB=$(find /tmp/r20_$TAG -name "*.db" | head -1)
python3 $R/tools/step_dispatches.py "$DB" 0.8 > $O/r20_dispatches.txt
rm -rf /tmp/r20_$TAG
echo "r20 trace ok"
