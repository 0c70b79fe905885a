#!/bin/bash
# One GPU call's worth of profiling for a build: kernel trace + PMC passes of the
# headline (rmat-cc), config-2 (RMAT-20), bipartiteness and ingest bench steps, summarised ON THE BOX
# (tools/rocprof_summary.py) so that only the small summaries come back: the raw
# rocprofv3 databases of three workloads exceed gpurun's 64 MiB return limit.
# Output: gpurun_out/profiles_<tag>/ (copy into profiles/ in the container).
# Usage (GPU box, repo root): bash tools/profile_round.sh <tag>
set -u
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/profiles_$TAG
mkdir -p $O
cd $R
bash tools/rocprof_round.sh $TAG || exit 1
python3 tools/rocprof_summary.py gpurun_out/rocprof_$TAG $TAG 3 || exit 1
bash tools/rocprof_round.sh ${TAG}_r20 --scale 20 --warmup 1 || exit 1
python3 tools/rocprof_summary.py gpurun_out/rocprof_${TAG}_r20 ${TAG}_r20 3 --workload rmat20 || exit 1
bash tools/pmc_workload.sh ${TAG}_bip bip || exit 1
python3 tools/rocprof_summary.py gpurun_out/rocprof_${TAG}_bip ${TAG}_bip 3 --workload bip || exit 1
bash tools/pmc_workload.sh ${TAG}_ing ingest || exit 1
python3 tools/rocprof_summary.py gpurun_out/rocprof_${TAG}_ing ${TAG}_ing 3 --workload ingest || exit 1
cp profiles/${TAG}_rocprof_summary.* profiles/${TAG}_r20_rocprof_summary.* profiles/${TAG}_bip_rocprof_summary.* \
   profiles/${TAG}_ing_rocprof_summary.* profiles/pmc_fold_traffic.json profiles/pmc_r20_traffic.json \
   profiles/pmc_bip_traffic.json profiles/pmc_ingest_traffic.json $O/ || exit 1
rm -rf gpurun_out/rocprof_$TAG gpurun_out/rocprof_${TAG}_r20 gpurun_out/rocprof_${TAG}_bip gpurun_out/rocprof_${TAG}_ing
echo "profiles in $O"
