#!/bin/bash
# Tracked-fold tax A/B: the delta-tracking tests, then rank 0's replayed
# exchange at N = 8 (tools/rank_replay.py, lag 2) with wave-aggregated record appends (default
# build) and with one append atomic per record (lib_nowave, GS_WAVE_APPEND=0).
set -u
O=gpurun_out/track_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_group.py tests/test_gpu_group_emulated.py tests/test_gpu_distributed.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for r in 1 2; do for v in default nowave; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  timeout -k 10 240 python -u tools/rank_replay.py --ranks 8 --lag 2 --reps 3 > $O/replay_${v}_$r.txt 2>&1 || { tail -5 $O/replay_${v}_$r.txt; exit 1; }
  echo "== $v ($r)"; grep -E "rank 0 alone|records sent|projected" $O/replay_${v}_$r.txt | cut -c1-220
done; done
# records per pass vs the ramp (more 2^20-edge exchanges while most vertices are new) and the data lag
unset GS_LIB_VARIANT
for cfg in "2 22" "2 24" "1 22" "1 24"; do
  set -- $cfg
  timeout -k 10 240 python -u tools/rank_replay.py --ranks 8 --lag $1 --ramp-log2 $2 --reps 2 > $O/replay_lag$1_ramp$2.txt 2>&1 || { tail -5 $O/replay_lag$1_ramp$2.txt; exit 1; }
  echo "== lag $1 ramp 2^$2"; grep -E "rank 0 alone|records sent|projected" $O/replay_lag$1_ramp$2.txt | cut -c1-220
done
