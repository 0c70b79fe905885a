#!/bin/bash
# Round 5: the ingest look-back variants on one box, interleaved (product = self-count code + 16-B fallback;
# ingnsc = no self-count code; ingold = round 4's look-back), then the product with the self-count at 1 us.
set -o pipefail
O=gpurun_out/${1:-r05j}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in base ingnsc ingold; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/ing_${v}_$r.json')); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'))" | tee -a $O/summary.txt
  done
done
