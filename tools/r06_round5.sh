#!/bin/bash
# Round-6: GPU suite after the capacity-wait and exact-count changes; configs 2/4/3, one-rank
# exchange lines; config-2 step dispatches; the N = 8 bulk replay with 32 HW queues (each rank's
# lanes on queues of their own) and the label forest's fold counters (debug build).
set -o pipefail
TAG=${1:-r06k}
R=$GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_ordering.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/gpu_tests_ordering.txt 2>&1 || { echo "ordering tests failed"; tail -30 $O/gpu_tests_ordering.txt; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --scale 20 --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass \
    > $O/bench_r20_$i.json 2> $O/bench_r20_$i.err || { echo "r20 rc=$?"; tail $O/bench_r20_$i.err; exit 1; }
  timeout -k 10 200 python -u bench.py --workload bip --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass \
    > $O/bench_bip_$i.json 2> $O/bench_bip_$i.err || { echo "bip rc=$?"; tail $O/bench_bip_$i.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-profile-pass > $O/bench.json 2> $O/bench.err \
  || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass \
  > $O/bench_exch.json 2> $O/bench_exch.err || { echo "exch rc=$?"; tail $O/bench_exch.err; exit 1; }
timeout -k 10 300 python -u bench.py --exchange --combine partitioned --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_part1.json 2> $O/bench_part1.err || { echo "bench part rc=$?"; tail -20 $O/bench_part1.err; exit 1; }
timeout -k 10 120 python -u tools/sync_check.py > $O/sync_check.txt 2>&1 || { echo "sync check rc=$?"; tail $O/sync_check.txt; exit 1; }
cat $O/sync_check.txt
grep -h '^{' $O/bench_r20_*.json $O/bench_bip_*.json $O/bench.json $O/bench_exch.json $O/bench_part1.json | cut -c1-170
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/r20_$TAG -o run -- python3 $R/bench.py --scale 20 --steps 3 --warmup 1 \
  --profile-only --no-profile-pass --no-cpu-baseline > $R/$O/r20_trace.log 2>&1 || { echo "r20 trace rc=$?"; exit 1; }
python3 $R/tools/step_dispatches.py $(find /tmp/r20_$TAG -name "*.db" | head -1) 0.8 > $R/$O/r20_dispatches.txt
rm -rf /tmp/r20_$TAG
cd $R
tail -45 $O/r20_dispatches.txt
GPU_MAX_HW_QUEUES=32 timeout -k 10 600 python -u tools/part_replay.py --ranks 8 --out $O/replay_w0_q32.json \
  > $O/replay_w0_q32.log 2>&1 || { echo "replay rc=$?"; tail -20 $O/replay_w0_q32.log; exit 1; }
python3 - $O/replay_w0_q32.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: v for k, v in d.items() if k != "per_rank"})
for x in d["per_rank"]:
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items() if k.endswith("_ms") or k == "pairs_sent"})
PY
GS_LIB_VARIANT=debug timeout -k 10 600 python -u tools/part_replay.py --ranks 8 --forest-counters \
  > $O/replay_forest_dbg.log 2>&1 || { echo "debug replay rc=$?"; tail -20 $O/replay_forest_dbg.log; exit 1; }
grep "label forest counters" $O/replay_forest_dbg.log
