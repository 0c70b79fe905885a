#!/bin/bash
# A/B of experiment builds on one GPU box (run from the repo root on the box):
# every variant library (gelly-streaming_amd/lib_<v>/, `make variant V=<v> VFLAGS=...`;
# "base" = the product build) runs the same bench lines, interleaved twice, into
# gpurun_out/variant_ab/<tag>/. A bench line that fails ends the run (no retries).
# Usage: bash tools/variant_ab.sh <tag> "<v1> <v2> ..." "<bench args 1>" ["<bench args 2>" ...]
set -u
TAG=$1; VARIANTS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/variant_ab/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in $VARIANTS; do
    i=0
    for a in "$@"; do
      i=$((i + 1))
      if [ "$v" = base ]; then env=""; else env="GS_LIB_VARIANT=$v"; fi
      f=$O/${v}_${i}_rep$rep.json
      env $env timeout -k 10 240 python bench.py $a > $f 2> $O/${v}_${i}_rep$rep.err || { echo "$v [$a] failed rc=$?"; exit 1; }
      echo "$v rep$rep [$a]: $(python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); c=d['config']; print(d['value'], d['ms_per_step'], c.get('p50_us'), c.get('p99_us'))")"
    done
  done
done
