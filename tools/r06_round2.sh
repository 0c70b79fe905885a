#!/bin/bash
# Round-6 check after the fence-free owner step and the label pass on the last lane: GPU suite,
# configs 2 / 3 / 4 lines (config 3 twice, config 2 three times: box noise), the partitioned
# one-rank line, a kernel trace of that line, and the RMAT-26 N = 8 partitioned replay.
set -o pipefail
TAG=${1:-r06h}
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --scale 20 --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass \
    > $O/bench_r20_$i.json 2> $O/bench_r20_$i.err || { echo "r20 rc=$?"; tail $O/bench_r20_$i.err; exit 1; }
done
timeout -k 10 200 python -u bench.py --workload bip --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass \
  > $O/bench_bip.json 2> $O/bench_bip.err || { echo "bip rc=$?"; tail $O/bench_bip.err; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-profile-pass > $O/bench_$i.json 2> $O/bench_$i.err \
    || { echo "bench rc=$?"; tail $O/bench_$i.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --exchange --combine partitioned --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_part1.json 2> $O/bench_part1.err || { echo "bench part rc=$?"; tail -20 $O/bench_part1.err; exit 1; }
grep -h '^{' $O/bench_r20_*.json $O/bench_bip.json $O/bench_?.json $O/bench_part1.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_part1 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --exchange --combine partitioned --steps 2 --warmup 1 --no-cpu-baseline \
  --no-profile-pass > $GRAFT_REPO_ROOT/$O/prof_part1.log 2>&1 || { echo "prof rc=$?"; exit 1; }
cd $GRAFT_REPO_ROOT
find $O/prof_part1 -name "*kernel_stats.csv" | head -1 | xargs -I{} head -25 {}
timeout -k 10 600 python -u tools/part_replay.py --ranks 8 --out $O/replay_bulk.json > $O/replay_bulk.log 2>&1 \
  || { echo "replay rc=$?"; tail -20 $O/replay_bulk.log; exit 1; }
python - $O/replay_bulk.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: v for k, v in d.items() if k != "per_rank"})
PY
