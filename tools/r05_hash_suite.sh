#!/bin/bash
# Round 5: the GPU suite on the line-grouped hash build, then bip / RMAT-20 against the plain hash (lib_hplain).
set -o pipefail
O=gpurun_out/${1:-r05v}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -2 $O/gpu_tests.txt | tee -a $O/summary.txt
[ $rc -eq 0 ] || exit $rc
VARIANT=hplain WORKLOADS="bip r20" ROUNDS=3 bash tools/r05_variant_ab.sh ${1:-r05v}
