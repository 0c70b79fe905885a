#!/bin/bash
# rocprofv3 kernel trace of ONLY the roofline's serialised pass (bench.py --steps 0 --profile-only --profile-serial):
# its k_fold average is the per-launch duration the bench line's `fold_avg_us` reports (HIP events), so the two can be
# compared directly (the pipelined step's trace overlaps dispatches). Args: extra bench args (e.g. --scale 20).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/serial_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
N=$(echo "$*" | tr -c 'a-z0-9' '_')
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/st_$N -o run -- python3 $R/bench.py --steps 0 --warmup 0 --profile-only --profile-serial --no-cpu-baseline "$@" > $O/log_$N.txt 2>&1 || { echo "trace failed"; tail -5 $O/log_$N.txt; exit 1; }
DB=$(find /tmp/st_$N -name "*.db" | head -1)
python3 $R/tools/timeline.py "$DB" 0 > $O/timeline_$N.txt
grep fold_avg_us $O/log_$N.txt
head -6 $O/timeline_$N.txt
rm -rf /tmp/st_$N
