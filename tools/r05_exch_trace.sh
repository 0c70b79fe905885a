#!/bin/bash
# Round 5: where the one-rank exchange step's extra time goes: kernel traces of one timed step
# of bench.py --exchange and of the plain pass (per-kernel totals, busy/idle, own-fold gaps), then the exchange
# line itself (phases).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r05g}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in exch plain; do
  A="--steps 1 --warmup 1 --profile-only --no-cpu-baseline --no-profile-pass"
  [ $v = exch ] && A="$A --exchange"
  timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/xk_$v -o run -- python3 $R/bench.py $A > $O/log_$v.txt 2>&1 || { echo "trace $v failed"; tail -5 $O/log_$v.txt; exit 1; }
  DB=$(find /tmp/xk_$v -name "*.db" | head -1)
  python3 $R/tools/timeline.py "$DB" 0 > $O/timeline_$v.txt || exit 1
  mkdir -p $O/db_$v && cp "$DB" $O/db_$v/ 
  echo "== $v"; head -16 $O/timeline_$v.txt; tail -1 $O/timeline_$v.txt
done
cd $R
timeout -k 10 300 python3 bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/bench_exch.json 2> $O/bench_exch.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_exch.json')); print('exch', d['ms_per_step'], d['config']['exchange_phases'])"
