#!/bin/bash
# GPU test suite (one pytest process), smoke, and the default bench line, each under its own
# time limit; stops at the first failure. Usage (repo root on the GPU box): bash tools/gpu_suite.sh <tag>
set -o pipefail
TAG=${1:-r06a}
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt
[ $rc -eq 0 ] || { echo "gpu tests rc=$rc"; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo "smoke failed"; cat $O/smoke.txt; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
cat $O/bench.json
