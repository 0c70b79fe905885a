#!/bin/bash
# Round 5: (1) the product look-back (4-B fallback, inline) against round 4's look-back (ingold), interleaved;
# (2) the ingest parity tests; (3) the one-rank exchange step with and without the combine ramp.
set -o pipefail
O=gpurun_out/${1:-r05l}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in base ingold; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/ing_${v}_$r.json')); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'))" | tee -a $O/summary.txt
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ingest.py > $O/ingest_tests.txt 2>&1 || exit 1
tail -1 $O/ingest_tests.txt | tee -a $O/summary.txt
for r in 1 2; do
  for ramp in 22 0; do
    timeout -k 10 300 python bench.py --exchange --ramp-log2 $ramp --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/exch_ramp${ramp}_$r.json 2> $O/exch_ramp${ramp}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/exch_ramp${ramp}_$r.json')); print('exch ramp$ramp r$r', d['ms_per_step'], json.dumps(d['config'].get('exchange_phases')))" | tee -a $O/summary.txt
  done
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/plain.json 2> $O/plain.err || exit 1
python -c "import json; d=json.load(open('$O/plain.json')); print('plain', d['ms_per_step'])" | tee -a $O/summary.txt
