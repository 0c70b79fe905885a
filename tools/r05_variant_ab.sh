#!/bin/bash
# Round 5: bench lines of several workloads, default build vs lib_$VARIANT, interleaved, ROUNDS rounds:
# ms/step (or the latency line's p50/p99) and each line's own checks.
set -o pipefail
O=gpurun_out/${1:-vab}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in $(seq 1 ${ROUNDS:-2}); do for w in ${WORKLOADS:-bip r20 n1 er}; do for v in default $VARIANT; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  case $w in bip) A="--workload bip";; r20) A="--scale 20";; n1) A="--steps 10 --warmup 2";; er) A="--workload er-latency";; esac
  timeout -k 10 300 python bench.py $A --no-cpu-baseline > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail -5 $O/${w}_${v}_$r.err; exit 1; }
  python - "$O/${w}_${v}_$r.json" "$w $v $r" <<'PY' | tee -a $O/summary.txt
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = l.get("config", {})
chk = {k: v for k, v in c.items() if k in ("self_check", "parity", "gpu_equals_reference", "diverges", "oracle_exact")}
extra = {k: l[k] for k in ("p50_us", "p99_us") if k in l}
for k in ("p50_us", "p99_us", "latency_p50_us", "latency_p99_us"):
    if k in c: extra[k] = c[k]
print(sys.argv[2], l["ms_per_step"], json.dumps(extra), json.dumps(chk)[:300])
PY
done; done; done
