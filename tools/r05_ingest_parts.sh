#!/bin/bash
# Round 5: ingest parse-kernel variants (VARIANTS, "base" = lib/), interleaved, two rounds: wall ms, kernel-rated
# and wall-rated roofline fractions, the kernel's event-timed us, parity.
set -o pipefail
O=gpurun_out/${1:-r05n}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in ${VARIANTS:-base pfloor pnolb pnolbfl}; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$O/ing_${v}_$r.json').read().splitlines()[-1]); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'), r.get('kernel_avg_us'), 'parity', d['config']['parity'])" | tee -a $O/summary.txt
  done
done
