#!/bin/bash
# One-rank RCCL exchange step (bench.py --exchange) by data lag (GS_GROUP_DATA_LAG) and combine ramp, two rounds.
set -u
O=gpurun_out/exch_ab
mkdir -p $O
for r in 1 2; do for cfg in "2 22" "2 24" "1 22" "1 24"; do
  set -- $cfg
  GS_GROUP_DATA_LAG=$1 timeout -k 10 240 python bench.py --exchange --ramp-log2 $2 --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/lag$1_ramp$2_$r.json 2> $O/lag$1_ramp$2_$r.err || { tail -5 $O/lag$1_ramp$2_$r.err; exit 1; }
  python -c "
import json; l=json.loads(open('$O/lag$1_ramp$2_$r.json').read().strip().splitlines()[-1]); c=l['config']
print('lag $1 ramp 2^$2', l['ms_per_step'], {k: c[k] for k in c if 'phase' in k or 'record' in k or 'sent' in k})"
done; done
