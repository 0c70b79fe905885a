#!/bin/bash
# Round 5: the ingest look-back's bounded self-count (GS_PARSE_SELFCOUNT_US) and the RCCL channel cap on the
# one-rank exchange step (--rccl-max-channels), A/B on one box; the ingest tests first.
set -o pipefail
O=gpurun_out/${1:-r05h}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -x -v --timeout 120 --timeout-method thread > $O/ingest_tests.txt 2>&1
rc=$?; tail -2 $O/ingest_tests.txt; [ $rc = 0 ] || exit $rc
for r in 1 2; do
  for sc in off 1 3 10; do
    if [ $sc = off ]; then E="X=1"; else E="GS_PARSE_SELFCOUNT_US=$sc"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${sc}_$r.json 2> $O/ing_${sc}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/ing_${sc}_$r.json')); r=d['roofline']; print('ingest sc=$sc r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'))" | tee -a $O/summary.txt
  done
done
for ch in 0 1 2 4; do
  timeout -k 10 300 python bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass --rccl-max-channels $ch > $O/exch_ch$ch.json 2> $O/exch_ch$ch.err || exit 1
  python -c "import json; L=[l for l in open('$O/exch_ch$ch.json') if l.startswith('{')]; d=json.loads(L[-1]); print('exch ch=$ch', d['ms_per_step'], d['config']['rccl'])" | tee -a $O/summary.txt
done
