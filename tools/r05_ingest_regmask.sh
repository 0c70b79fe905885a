#!/bin/bash
# Round 5: '\n' masks from the staging registers (product) against masks from LDS (pnoreg), interleaved; the
# look-back statistics build (plbs: per-tile phase times); the ingest parity tests.
set -o pipefail
O=gpurun_out/${1:-r05q}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in ${VARIANTS:-base pnoreg}; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$O/ing_${v}_$r.json').read().splitlines()[-1]); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'), r.get('kernel_avg_us'), 'parity', d['config']['parity'])" | tee -a $O/summary.txt
  done
done
GS_LIB_VARIANT=plbs timeout -k 10 240 python bench.py --workload ingest --steps 5 --warmup 2 --no-cpu-baseline > $O/plbs.json 2> $O/plbs.err || exit 1
grep -E "LBSTATS|LBPHASES" $O/plbs.err | head -4 | tee -a $O/summary.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ingest.py > $O/ingest_tests.txt 2>&1 || exit 1
tail -1 $O/ingest_tests.txt | tee -a $O/summary.txt
