#!/bin/bash
# Ingest A/B on the GPU box: the parse modes of gs_parse_edges_device (GS_PARSE_MODE:
# 2 = pipelined two-pass, 1 = one pass with look-back, 0 = plain two-pass), after the tests.
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ing_tests.txt 2>&1 || { tail -20 gpurun_out/ing_tests.txt; exit 1; }
tail -1 gpurun_out/ing_tests.txt
for r in 1 2; do for v in ${MODES:-2 1 0}; do for tk in ${TICKETS:-1}; do
  GS_PARSE_TICKET=$tk GS_PARSE_MODE=$v timeout -k 10 120 python bench.py --workload ingest --steps 20 --warmup 3 > gpurun_out/ing_ab.json 2>gpurun_out/ing_err.txt || exit 1
  python -c "import json; l=json.loads(open('gpurun_out/ing_ab.json').read().strip().splitlines()[-1]); print('mode $v ticket $tk', l['ms_per_step'], l['roofline']['frac'], l['config']['parity'])"
done; done; done
