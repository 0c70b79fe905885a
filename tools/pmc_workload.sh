#!/bin/bash
# Kernel trace + PMC passes of one bench workload (each PMC group its own rocprofv3 run;
# counters are never combined with tracing domains), on the GPU box from the repo root.
# Usage: bash tools/pmc_workload.sh <tag> <workload> [bench args...]
#   workload rmat-cc | bip : the fold's traffic passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss,
#                            fabric read requests)
#   workload ingest        : the same + SQ passes (VALU / LDS activity, LDS bank conflicts)
# Then, in the container: python tools/rocprof_summary.py gpurun_out/rocprof_<tag> <tag> <pipeline> [batch] --workload <w>
set -u
TAG=$1; W=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rocprof_$TAG
mkdir -p $OUT
ARGS="--workload $W --steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass --profile-only $*"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace ok"
PASSES=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum")
if [ "$W" = "ingest" ]; then
  PASSES+=("SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE GRBM_COUNT")
fi
for P in "${PASSES[@]}"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-60)
  timeout -s KILL 180 rocprofv3 --pmc $P -d $OUT/pmc_$N -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_$N.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc $P failed rc=$rc"; tail -3 $OUT/pmc_$N.log; case $rc in 137|124|134|139) exit $rc;; esac; else echo "pmc $P ok"; fi
done
