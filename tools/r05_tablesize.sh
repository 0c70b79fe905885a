#!/bin/bash
# Per-batch k_fold time against the table's size (no slack sizing, serial folds: the exact vertex count after
# every fold keeps the table at the hint's size): configs 2 and 4 at 2^21 .. 2^24 slots.
set -o pipefail
O=gpurun_out/${1:-r05e}
mkdir -p $O
export PYTHONUNBUFFERED=1
for h in 19 20 21 22; do
  GS_SLACK_GROW=0 GS_YOUNG_HEAD_LOG2=0 timeout -k 10 120 python tools/fold_stats.py r20 --hint-log2 $h > $O/r20_h$h.txt 2>&1 || exit 1
  GS_SLACK_GROW=0 GS_YOUNG_HEAD_LOG2=0 timeout -k 10 120 python tools/fold_stats.py bip --hint-log2 $h > $O/bip_h$h.txt 2>&1 || exit 1
done
for f in $O/*_h*.txt; do echo "$f $(grep '^#' $f) sum_us $(awk 'NR>2 && $1 ~ /^[0-9]+$/ {s+=$2} END {print s}' $f) steady_us $(awk 'NR>2 && $1 ~ /^[0-9]+$/ && $1 >= 8 {s+=$2; n++} END {print s/n}' $f)"; done | tee $O/summary.txt
