#!/bin/bash
# Round-6: partitioned + group tests; the own-fold probe (tools/sync_check.py); the N = 8 bulk
# replay after the label forest's young head.
set -o pipefail
TAG=${1:-r06m}
O=gpurun_out/$TAG
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py tests/test_gpu_group_emulated.py tests/test_gpu_group.py \
  -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/gpu_tests.txt | head -20
tail -2 $O/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/sync_check.py > $O/sync_check.txt 2>&1 || { echo "probe rc=$?"; tail $O/sync_check.txt; exit 1; }
cat $O/sync_check.txt
timeout -k 10 600 python -u tools/part_replay.py --ranks 8 --out $O/replay_w0.json > $O/replay_w0.log 2>&1 \
  || { echo "replay rc=$?"; tail -20 $O/replay_w0.log; exit 1; }
python3 - $O/replay_w0.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print({k: v for k, v in d.items() if k != "per_rank"})
for x in d["per_rank"]:
    print({k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items() if k.endswith("_ms") or k == "pairs_sent"})
PY
