#!/bin/bash
# Round-end evidence for one build, run on the GPU box from the repo root: the GPU test
# suite, smoke(), and one bench line per workload into gpurun_out/final_<tag>/.
# (Profile first with tools/rocprof_round.sh + tools/rocprof_summary.py so that the
# N=1 line's traffic comes from a profile of the same library.)
# Usage: bash tools/final_round.sh <tag>
set -u
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final_$TAG
mkdir -p $O
cd $R
step() {  # name, limit, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.out 2> $O/$n.err || { echo "$n failed rc=$?"; exit 1; }
  echo "$n ok"
}
step gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 300 python bench.py --steps 20 --warmup 2
step bench_r20 200 python bench.py --scale 20 --steps 20 --warmup 2
step bench_bip 120 python bench.py --workload bip --steps 10
step bench_er 120 python bench.py --workload er-latency --steps 1
step bench_ingest 120 python bench.py --workload ingest --steps 10
step bench_dropin 200 python bench.py --workload dropin
step bench_exch 200 python bench.py --exchange --steps 5 --no-cpu-baseline
