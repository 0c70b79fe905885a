#!/bin/bash
# Partitioned mode: its GPU tests, the one-rank RCCL bench line of the partitioned path, then
# the RMAT-26 N = 8 replays (tools/r06_replay.sh).
set -o pipefail
TAG=${1:-r06e}
O=gpurun_out/$TAG
bash tools/gpu_tests_sel.sh $TAG tests/test_gpu_partitioned.py || exit 1
timeout -k 10 300 python -u bench.py --exchange --combine partitioned --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_part1.json 2> $O/bench_part1.err || { echo "bench part rc=$?"; tail -20 $O/bench_part1.err; exit 1; }
cat $O/bench_part1.json
bash tools/r06_replay.sh $TAG
