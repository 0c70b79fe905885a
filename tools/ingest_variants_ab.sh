#!/bin/bash
# Ingest bench line over library variants (VARIANTS, "default" = lib/), two rounds: wall ms and the kernel's event-timed us.
set -u
O=gpurun_out/ingest_variants
mkdir -p $O
for r in 1 2; do for v in $VARIANTS; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  timeout -k 10 200 python bench.py --workload ingest --steps 20 --warmup 3 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
  python -c "import json; l=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); r=l['roofline']; print('$v $r', l['ms_per_step'], r['kernel_avg_us'], r['frac'], l['config']['parity'])"
done; done
