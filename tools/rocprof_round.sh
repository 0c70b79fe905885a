#!/bin/bash
# Kernel-trace + PMC passes of one bench step, at the bench's own default settings
# (pipeline depth 3), run on the GPU box from the repo root. Each PMC group is its own
# rocprofv3 run (counters are never combined with tracing domains).
# Usage: bash tools/rocprof_round.sh <tag> [bench args...]
# Then, in the container: python tools/rocprof_summary.py gpurun_out/rocprof_<tag> <tag> <pipeline>
set -u
TAG=${1:-r02}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rocprof_$TAG
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass --profile-only $*"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace ok"
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  N=$(echo $P | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/pmc_$N -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_$N.log 2>&1 || { echo "pmc $P failed rc=$?"; exit 1; }
  echo "pmc $P ok"
done
