#!/bin/bash
# Round-5 remote-row A/B: rank 0 of the N = 8 replay (tools/rank_replay.py --row-stats) for
# the product build and the variants: rt2/rt0 = re-read before the key CAS on the new parent's side only / on
# neither side of other replicas' rows; dir = direct hook of a freshly inserted larger-key endpoint under the other;
# sc1 = first probes as L1-bypassing loads. Then the config-2/4/3 bench lines of the variants that change plain folds.
# Then the GPU suite.
set -o pipefail
O=gpurun_out/${1:-r05d}
mkdir -p $O
export PYTHONUNBUFFERED=1
for v in base rt2 rt0 dir dir2 sc1 sc1r; do
  if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
  env $E timeout -k 10 200 python tools/rank_replay.py --row-stats --reps 2 --lag 2 > $O/replay_$v.txt 2>&1 || exit 1
  echo "$v $(grep 'row-stats rep 1 remote' $O/replay_$v.txt | sed 's/;.*//') | $(grep 'own tracked folds + takes' $O/replay_$v.txt)" | tee -a $O/summary.txt
done
for r in 1 2; do
  for v in base dir sc1; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    for w in r20 bip rmat26; do
      case $w in r20) A="--scale 20 --steps 30 --warmup 5";; bip) A="--workload bip --steps 30 --warmup 5";; rmat26) A="--steps 5 --warmup 2";; esac
      env $E timeout -k 10 240 python bench.py $A --no-cpu-baseline --no-profile-pass > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || exit 1
      python -c "import json; d=json.load(open('$O/${w}_${v}_$r.json')); print('${w}_${v}_$r', d['ms_per_step'])" | tee -a $O/summary.txt
    done
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
echo "rc=$rc"
exit $rc
