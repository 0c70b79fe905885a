#!/bin/bash
# Round 5: pending links (GS_PENDING_LINK, lib_pend): the GPU suite on the variant, the bench lines against the
# default build, and rank 0 of the N = 8 replay.
set -o pipefail
O=gpurun_out/${1:-r05p1}
mkdir -p $O
export PYTHONUNBUFFERED=1
GS_LIB_VARIANT=pend timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
tail -3 $O/gpu_tests.txt | tee -a $O/summary.txt
[ $rc -eq 0 ] || exit $rc
VARIANT=pend WORKLOADS="bip r20 n1 er" ROUNDS=2 bash tools/r05_variant_ab.sh ${1:-r05p1} || exit 1
GS_LIB_VARIANT=pend timeout -k 10 300 python tools/rank_replay.py --row-stats --reps 2 --lag 2 > $O/replay_pend.txt 2>&1 || exit 1
timeout -k 10 300 python tools/rank_replay.py --row-stats --reps 2 --lag 2 > $O/replay_default.txt 2>&1 || exit 1
grep -h "row-stats\|alone\|projected" $O/replay_pend.txt $O/replay_default.txt | tee -a $O/summary.txt
