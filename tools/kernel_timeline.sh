#!/bin/bash
# Kernel timeline (busy / idle / overlap) of a program under rocprofv3 --kernel-trace,
# summarised on the box; the trace database is deleted afterwards.
# Usage (repo root on the GPU box): bash tools/kernel_timeline.sh <tag> <skip_ms> <python script> [args...]
set -u
TAG=$1; SKIP=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ktl_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/ktl_$TAG -o run -- python3 "$@" > $OUT/log 2>&1 || { echo "trace failed rc=$?"; tail -5 $OUT/log; exit 1; }
DB=$(find /tmp/ktl_$TAG -name "*.db" | head -1)
python3 $R/tools/timeline.py "$DB" $SKIP > $OUT/timeline.txt
rm -rf /tmp/ktl_$TAG
cat $OUT/timeline.txt
