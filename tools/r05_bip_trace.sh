#!/bin/bash
# Round 5: per-dispatch kernel trace of the config-4 step (tools/step_dispatches.py) on this build.
set -u
TAG=${1:-r05w}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/bip_$TAG -o run -- python3 $R/bench.py --workload bip --steps 3 --warmup 1 --profile-only --no-profile-pass > $O/bip_trace.log 2>&1 || { echo "bip trace failed rc=$?"; exit 1; }
DB=$(find /tmp/bip_$TAG -name "*.db" | head -1)
python3 $R/tools/step_dispatches.py "$DB" 1.2 > $O/bip_dispatches.txt
python3 $R/tools/timeline.py "$DB" 0 > $O/bip_timeline.txt
echo "bip trace ok"
