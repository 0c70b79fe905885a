#!/bin/bash
# Round-6: partitioned tests after the pair set; one-rank partitioned line with a kernel table and
# its idle gaps; config-2 step dispatches; RMAT-26 N = 8 replays (bulk, 2^22-edge windows).
set -o pipefail
TAG=${1:-r06j}
R=$GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_group_emulated.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --exchange --combine partitioned --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_part1.json 2> $O/bench_part1.err || { echo "bench part rc=$?"; tail -20 $O/bench_part1.err; exit 1; }
grep -h '^{' $O/bench_part1.json | cut -c1-160
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p1_$TAG -o run -- python3 $R/bench.py --exchange --combine partitioned \
  --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass --profile-only > $R/$O/prof_part1.log 2>&1 \
  || { echo "prof rc=$?"; exit 1; }
DB=$(find /tmp/p1_$TAG -name "*.db" | head -1)
python3 $R/tools/kernel_table.py $DB 25 > $R/$O/part1_kernels.txt
python3 $R/tools/gaps.py $DB 60 25 > $R/$O/part1_gaps.txt
timeout -k 10 240 rocprofv3 --kernel-trace -d /tmp/r20_$TAG -o run -- python3 $R/bench.py --scale 20 --steps 3 --warmup 1 \
  --profile-only --no-profile-pass --no-cpu-baseline > $R/$O/r20_trace.log 2>&1 || { echo "r20 trace rc=$?"; exit 1; }
python3 $R/tools/step_dispatches.py $(find /tmp/r20_$TAG -name "*.db" | head -1) 0.8 > $R/$O/r20_dispatches.txt
rm -rf /tmp/p1_$TAG /tmp/r20_$TAG
cd $R
cat $O/part1_gaps.txt | head -15
tail -40 $O/r20_dispatches.txt
for M in 0 22; do
  timeout -k 10 600 python -u tools/part_replay.py --ranks 8 --window-log $M --out $O/replay_w$M.json > $O/replay_w$M.log 2>&1 \
    || { echo "replay rc=$?"; tail -20 $O/replay_w$M.log; exit 1; }
  python3 - $O/replay_w$M.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: v for k, v in d.items() if k != "per_rank"})
for x in d["per_rank"]:
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items() if k.endswith("_ms") or k == "pairs_sent"})
PY
done
