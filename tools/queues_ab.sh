#!/bin/bash
# One-rank RCCL exchange step and the plain pass with 4 vs 8 hardware queues per process (GPU_MAX_HW_QUEUES), two rounds.
set -u
O=gpurun_out/queues_ab
mkdir -p $O
for r in 1 2; do for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/exch_q${q}_$r.json 2> $O/exch_q${q}_$r.err || { tail -5 $O/exch_q${q}_$r.err; exit 1; }
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/n1_q${q}_$r.json 2> $O/n1_q${q}_$r.err || { tail -5 $O/n1_q${q}_$r.err; exit 1; }
  python -c "
import json
for w in ('exch', 'n1'):
    l = json.loads(open('$O/%s_q${q}_$r.json' % w).read().strip().splitlines()[-1]); p = l['config'].get('exchange_phases') or {}
    print('queues $q round $r', w, l['ms_per_step'], {k: p[k] for k in ('host_wait_counts_ms', 'stage_count_collective_ms') if k in p})"
done; done
