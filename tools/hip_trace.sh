#!/bin/bash
# Host-side HIP API cost of a program (rocprofv3 --hip-trace), summarised on the box;
# the trace database is deleted afterwards (too large to bring back).
# Usage (repo root on the GPU box): bash tools/hip_trace.sh <tag> <python script> [args...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/hiptr_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace -d /tmp/hiptr_$TAG -o run -- python3 "$@" > $OUT/log 2>&1 || { echo "trace failed rc=$?"; tail -5 $OUT/log; exit 1; }
DB=$(find /tmp/hiptr_$TAG -name "*.db" | head -1)
python3 $R/tools/hip_api_summary.py "$DB" 30 > $OUT/hip_api.txt
rm -rf /tmp/hiptr_$TAG
cat $OUT/hip_api.txt
