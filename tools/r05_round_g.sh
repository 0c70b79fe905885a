#!/bin/bash
# Round 5: GPU suite on the product build, then the one-rank exchange traces.
set -o pipefail
O=gpurun_out/${1:-r05g}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?; tail -2 $O/gpu_tests.txt; [ $rc = 0 ] || exit $rc
bash tools/r05_exch_trace.sh ${1:-r05g}
