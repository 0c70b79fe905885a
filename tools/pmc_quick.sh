#!/bin/bash
# Quick PMC comparison of k_fold variants: bash tools/pmc_quick.sh <tag> [env assignments...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
for kv in "$@"; do export "$kv"; done
OUT=$R/gpurun_out/pmcq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/a -o run -- python3 $R/bench.py $ARGS > $OUT/a.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/t -o run -- python3 $R/bench.py $ARGS > $OUT/t.log 2>&1 || exit 1
echo "pmc $TAG ok"
