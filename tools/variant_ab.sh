#!/bin/bash
# A/B of the default build against lib_<variant> (GS_LIB_VARIANT) on the bench lines named in WORKLOADS
# (bip, r20, er, n1), two rounds, one box. Usage: VARIANT=noreserve WORKLOADS="bip r20 er" bash tools/variant_ab.sh
set -u
O=gpurun_out/variant_ab
mkdir -p $O
for r in 1 2; do for v in default $VARIANT; do for w in $WORKLOADS; do
  if [ $v = default ]; then unset GS_LIB_VARIANT; else export GS_LIB_VARIANT=$v; fi
  case $w in
    bip) A="--workload bip";; r20) A="--scale 20";; er) A="--workload er-latency";; n1) A="--steps 5 --warmup 2";;
    ingest) A="--workload ingest";;
  esac
  timeout -k 10 300 python bench.py $A --no-cpu-baseline --no-profile-pass > $O/${w}_${v}_$r.json 2> $O/${w}_${v}_$r.err || { tail -5 $O/${w}_${v}_$r.err; exit 1; }
  python - $O/${w}_${v}_$r.json "$w $v $r" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c = l["config"]
extra = {k: c[k] for k in ("p50_us", "p99_us", "tail") if k in c}
print(sys.argv[2], l["ms_per_step"], l["value"], extra.get("tail", extra) if extra else "")
PY
done; done; done
