#!/bin/bash
# One-rank RCCL exchange step (bench.py --exchange) over several library variants (VARIANTS, "default" = lib/), two rounds.
set -u
O=gpurun_out/exch_variant
mkdir -p $O
for r in 1 2; do for v in $VARIANTS; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  timeout -k 10 240 python bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
  python -c "import json; l=json.loads(open('$O/${v}_$r.json').read().strip().splitlines()[-1]); print('$v $r', l['ms_per_step'])"
done; done
