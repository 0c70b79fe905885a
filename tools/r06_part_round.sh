#!/bin/bash
# Partitioned mode: its GPU tests, then the RMAT-26 N = 8 replays (tools/r06_replay.sh).
set -o pipefail
TAG=${1:-r06e}
bash tools/gpu_tests_sel.sh $TAG tests/test_gpu_partitioned.py || exit 1
bash tools/r06_replay.sh $TAG
