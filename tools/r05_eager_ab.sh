#!/bin/bash
# Round 5: eager data halves (GS_GROUP_EAGER, default on) -- the group tests, the one-rank exchange line eager vs the
# fixed lag 2, a kernel trace of the eager exchange step; and the ingest look-back variants (product = self-count
# code + 16-B fallback; ingnsc = no self-count code; ingold = round 4's look-back).
set -o pipefail
O=gpurun_out/${1:-r05i}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_group_emulated.py tests/test_gpu_ordering.py tests/test_gpu_configs_multi.py tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > $O/group_tests.txt 2>&1
rc=$?; tail -2 $O/group_tests.txt; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for e in 1 0; do
    GS_GROUP_EAGER=$e timeout -k 10 300 python bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/exch_e${e}_$r.json 2> $O/exch_e${e}_$r.err || exit 1
    python -c "import json; L=[l for l in open('$O/exch_e${e}_$r.json') if l.startswith('{')]; d=json.loads(L[-1]); p=d['config']['exchange_phases']; print('exch eager=$e r$r', d['ms_per_step'], 'wait', p['host_wait_counts_ms'], 'digest', d['config']['self_check']['digest_equals_single_gpu'])" | tee -a $O/summary.txt
  done
  for v in base ingnsc ingold; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/ing_${v}_$r.json')); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'))" | tee -a $O/summary.txt
  done
done
bash tools/r05_exch_trace.sh ${1:-r05i}_trace > /dev/null 2>&1 || echo "trace failed"
echo done
