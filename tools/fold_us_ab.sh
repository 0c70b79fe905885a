#!/bin/bash
# Serialised per-launch fold time (the bench's profile pass, HIP events) and step time: default vs lib_$VARIANT,
# on the bip and RMAT-20 lines, two rounds.
set -u
O=gpurun_out/fold_us_ab
mkdir -p $O
for r in 1 2; do for v in default $VARIANT; do for w in ${WORKLOADS:-bip r20}; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  case $w in bip) A="--workload bip";; r20) A="--scale 20";; n1) A="--steps 5 --warmup 2";; esac
  timeout -k 10 300 python bench.py $A --no-cpu-baseline > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail -5 $O/${w}_${v}_$r.err; exit 1; }
  python -c "import json; l=json.loads(open('$O/${w}_${v}_$r.json').read().strip().splitlines()[-1]); print('$w $v $r', l['ms_per_step'], l['roofline']['fold_avg_us'])"
done; done; done
