#!/bin/bash
# Round 5: the product look-back (round 4's loop + the 16-B fallback out of line) against round 4's
# look-back (ingold), interleaved on one box; then the ingest parity tests.
set -o pipefail
O=gpurun_out/${1:-r05k}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in base ingold; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/ing_${v}_$r.json')); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'))" | tee -a $O/summary.txt
  done
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ingest.py > $O/ingest_tests.txt 2>&1
