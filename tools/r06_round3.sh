#!/bin/bash
# Round-6 check: GPU suite; configs 2 / 4 / 3 after the slack revert; the partitioned one-rank
# line with its kernel table; the RMAT-26 N = 8 partitioned replay (bulk) with its kernel table.
set -o pipefail
TAG=${1:-r06i}
R=$GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
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
grep -h '^{' $O/bench_r20_*.json $O/bench_bip_*.json $O/bench.json $O/bench_exch.json $O/bench_part1.json | cut -c1-180
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/p1_$TAG -o run -- python3 $R/bench.py --exchange --combine partitioned \
  --steps 2 --warmup 1 --no-cpu-baseline --no-profile-pass > $R/$O/prof_part1.log 2>&1 || { echo "prof rc=$?"; exit 1; }
python3 $R/tools/kernel_table.py $(find /tmp/p1_$TAG -name "*.db" | head -1) 30 > $R/$O/part1_kernels.txt
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/rp_$TAG -o run -- python3 $R/tools/part_replay.py --ranks 8 \
  --out $R/$O/replay_bulk.json > $R/$O/replay_bulk.log 2>&1 || { echo "replay rc=$?"; tail -20 $R/$O/replay_bulk.log; exit 1; }
python3 $R/tools/kernel_table.py $(find /tmp/rp_$TAG -name "*.db" | head -1) 40 > $R/$O/replay_kernels.txt
rm -rf /tmp/p1_$TAG /tmp/rp_$TAG
cd $R
head -20 $O/part1_kernels.txt
head -30 $O/replay_kernels.txt
python3 - $O/replay_bulk.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: v for k, v in d.items() if k != "per_rank"})
for x in d["per_rank"]:
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items() if k.endswith("_ms")})
PY
