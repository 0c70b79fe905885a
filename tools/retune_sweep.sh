#!/bin/bash
# Exchange-loop time vs the retune period / header lag (GS_GROUP_RETUNE, GS_GROUP_LAG):
# one rank through RCCL (bench.py --exchange) and the mean all-gather capacity.
# Usage (GPU box, repo root): bash tools/retune_sweep.sh
for cfg in "4 4" "2 2" "1 1" "1 2"; do
  set -- $cfg
  r=$(GS_GROUP_RETUNE=$1 GS_GROUP_LAG=$2 GS_GROUP_HOSTPROF=1 timeout -k 10 150 python bench.py --no-cpu-baseline --no-profile-pass --exchange --steps 3 2>&1 | grep -oE "ms_per_step\": [0-9.]*|mean cap [0-9]*" | tail -2 | tr '\n' ' ') || { echo "[$cfg] failed"; exit 1; }
  echo "[retune $1 lag $2] $r"
done
