#!/bin/bash
# Round-5: settled inserts (GS_SETTLE, lib_settle) -- the GPU suite on the variant, then rank 0 of the N = 8 replay
# and the config-2/4/3 bench lines, product vs settle, two interleaved rounds; then the table-size probe.
set -o pipefail
O=gpurun_out/${1:-r05f}
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in base settle; do
  if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
  env $E timeout -k 10 200 python tools/rank_replay.py --row-stats --reps 2 --lag 2 > $O/replay_$v.txt 2>&1 || exit 1
  echo "$v $(grep 'row-stats rep 1 remote' $O/replay_$v.txt | sed 's/;.*//') | $(grep 'remote rows (0.35' $O/replay_$v.txt)" | tee -a $O/summary.txt
done
for r in 1 2; do
  for v in base settle; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    for w in r20 bip rmat26; do
      case $w in r20) A="--scale 20 --steps 30 --warmup 5";; bip) A="--workload bip --steps 30 --warmup 5";; rmat26) A="--steps 5 --warmup 2";; esac
      env $E timeout -k 10 240 python bench.py $A --no-cpu-baseline --no-profile-pass > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || exit 1
      python -c "import json; d=json.load(open('$O/${w}_${v}_$r.json')); print('${w}_${v}_$r', d['ms_per_step'])" | tee -a $O/summary.txt
    done
  done
done
for v in base settle; do
  if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
  env $E timeout -k 10 120 python tools/fold_stats.py bip > $O/bip_times_$v.txt 2>&1 || exit 1
  env $E timeout -k 10 120 python tools/fold_stats.py r20 > $O/r20_times_$v.txt 2>&1 || exit 1
done
bash tools/r05_tablesize.sh ${1:-r05f}_ts || exit 1
GS_LIB_VARIANT=settle timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_settle.txt 2>&1
rc=$?; tail -2 $O/gpu_tests_settle.txt
echo "rc=$rc"
