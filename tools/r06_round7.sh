#!/bin/bash
# Round-6: GPU suite after the wait changes; config 2/4/3/5 lines, one-rank exchange lines; the
# N = 8 bulk replay (own folds timed by Summary.sync() must now match a kernel-based wait).
set -o pipefail
TAG=${1:-r06q}
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
step() {  # name, limit, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "$n rc=$?"; tail $O/$n.err; exit 1; }
}
step bench_r20_1 200 --scale 20 --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass
step bench_r20_2 200 --scale 20 --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass
step bench_bip_1 200 --workload bip --steps 20 --warmup 3 --no-cpu-baseline --no-profile-pass
step bench 300 --no-cpu-baseline --no-profile-pass
step bench_exch 300 --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass
step bench_part1 300 --exchange --combine partitioned --steps 5 --warmup 2 --no-cpu-baseline
step bench_er 200 --workload er-latency --steps 1
grep -h '^{' $O/bench*.json | cut -c1-150
timeout -k 10 600 python -u tools/part_replay.py --ranks 8 --out $O/replay_w0.json > $O/replay_w0.log 2>&1 \
  || { echo "replay rc=$?"; tail -20 $O/replay_w0.log; exit 1; }
python3 - $O/replay_w0.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: v for k, v in d.items() if k != "per_rank"})
for x in d["per_rank"]:
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items() if k.endswith("_ms")})
PY
