#!/bin/bash
# Round 5: config 4 on the line-grouped hash: young-table head sizes (GS_YOUNG_HEAD_LOG2), interleaved, three rounds.
set -o pipefail
O=gpurun_out/${1:-r05x}
mkdir -p $O
for r in 1 2 3; do for h in 14 0 17 19; do
  E="GS_YOUNG_HEAD_LOG2=$h"
  env $E timeout -k 10 200 python bench.py --workload bip --steps 20 --no-cpu-baseline > $O/bip_${h}_$r.json 2> $O/bip_${h}_$r.err || exit 1
  python -c "import json; l=json.loads(open('$O/bip_${h}_$r.json').read().strip().splitlines()[-1]); print('bip head $h r$r', l['ms_per_step'], l['config']['verdict_parity'])" | tee -a $O/summary.txt
done; done
