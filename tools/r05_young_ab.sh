#!/bin/bash
# Round-5 young-table A/B: configs 2 (RMAT-20) and 4 (bipartite) bench lines for the product
# build, the young head split (GS_YOUNG_HEAD_LOG2), the insert re-read (lib_ttas) and 4 combine
# rounds (lib_cr4); two interleaved rounds. Also the product's serial per-batch times.
set -o pipefail
O=gpurun_out/${1:-r05b}
mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name, env..., -- bench args
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 180 python bench.py "$@" --no-cpu-baseline --no-profile-pass > $O/$name.json 2> $O/$name.err || return 1
  python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['ms_per_step'])" | tee -a $O/summary.txt
}
for r in 1 2; do
  for w in r20 bip; do
    if [ $w = r20 ]; then A="--scale 20 --steps 30 --warmup 5"; else A="--workload bip --steps 30 --warmup 5"; fi
    run ${w}_base_$r X=1 -- $A &&
    run ${w}_head12_$r GS_YOUNG_HEAD_LOG2=12 -- $A &&
    run ${w}_head14_$r GS_YOUNG_HEAD_LOG2=14 -- $A &&
    run ${w}_head16_$r GS_YOUNG_HEAD_LOG2=16 -- $A &&
    run ${w}_ttas_$r GS_LIB_VARIANT=ttas -- $A &&
    run ${w}_cr4_$r GS_LIB_VARIANT=cr4 -- $A || exit 1
  done
done
timeout -k 10 120 python tools/fold_stats.py r20 > $O/r20_times.txt 2>&1 &&
GS_YOUNG_HEAD_LOG2=14 timeout -k 10 120 python tools/fold_stats.py r20 > $O/r20_times_head14.txt 2>&1
echo "rc=$?"
