#!/bin/bash
# A selection of the GPU tests (one pytest process, no -x: every selected test reports).
# Usage: bash tools/gpu_tests_sel.sh <tag> <pytest args...>
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread "$@" > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/gpu_tests.txt | tail -40
tail -3 $O/gpu_tests.txt
exit $rc
