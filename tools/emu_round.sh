#!/bin/bash
# Emulated N-rank exchange on one GPU: inflation at the default hardware-queue count,
# then kernel traces of the N=2/4/8 runs split into phases. gpurun_out/emu/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/emu
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/emulated_scaling.py --ranks 1,2,4,8 --reps 2 > $OUT/q4.txt 2>&1
for N in 2 4 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr$N -o run -- python3 $R/tools/emulated_scaling.py --ranks $N --reps 1 > $OUT/tr$N.log 2>&1
  python3 $R/tools/exchange_breakdown.py $OUT/tr$N --ranks $N --passes 2 > $OUT/breakdown$N.json
  rm -rf $OUT/tr$N
done
cat $OUT/q4.txt $OUT/breakdown*.json
