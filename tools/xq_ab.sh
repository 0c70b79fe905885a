#!/bin/bash
# A/B of the cross-queue hand-off: event waits (lib/) vs memory-value waits (lib_xqv/, built with
# make variant V=xqv VFLAGS=-DGS_XQ_VALUE=1) on configs 2 and 4, after the hand-off probe and a
# parity pass of the variant.
set -o pipefail
O=gpurun_out/xq; mkdir -p $O
timeout -k 10 60 ./tools/xq_probe 200 > $O/probe.txt 2>&1 || { echo "probe failed rc=$?"; exit 1; }
cat $O/probe.txt
GS_LIB_VARIANT=xqv timeout -k 10 400 python -u -m pytest tests/test_gpu_ordering.py tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { echo "variant tests failed rc=$?"; tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for i in 1 2; do
  for v in base xqv; do
    if [ $v = xqv ]; then export GS_LIB_VARIANT=xqv; else unset GS_LIB_VARIANT; fi
    timeout -k 10 200 python bench.py --scale 20 --steps 20 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/${v}_r20_$i.json 2> $O/${v}_r20_$i.err || { echo "r20 $v failed rc=$?"; exit 1; }
    timeout -k 10 200 python bench.py --workload bip --steps 10 --no-cpu-baseline --no-profile-pass > $O/${v}_bip_$i.json 2> $O/${v}_bip_$i.err || { echo "bip $v failed rc=$?"; exit 1; }
    python3 -c "import json,sys
for f in sys.argv[1:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d['ms_per_step'])" $O/${v}_r20_$i.json $O/${v}_bip_$i.json
  done
done
