#!/bin/bash
# The GPU test suite (one pytest process), then the new round-5 tests' output kept.
set -o pipefail
O=gpurun_out/${1:-r05c}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
echo "rc=$rc"
exit $rc
