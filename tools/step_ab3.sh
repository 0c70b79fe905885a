#!/bin/bash
# Step time, default vs lib_$VARIANT, interleaved, 3 rounds (bench lines without profile pass / CPU baseline).
set -u
O=gpurun_out/step_ab3
mkdir -p $O
for r in 1 2 3; do for v in default $VARIANT; do for w in ${WORKLOADS:-n1 r20 bip}; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  case $w in bip) A="--workload bip";; r20) A="--scale 20";; n1) A="--steps 10 --warmup 2";; esac
  timeout -k 10 300 python bench.py $A --no-cpu-baseline --no-profile-pass > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail -5 $O/${w}_${v}_$r.err; exit 1; }
  python -c "import json; l=json.loads(open('$O/${w}_${v}_$r.json').read().strip().splitlines()[-1]); print('$w $v $r', l['ms_per_step'])"
done; done; done
