#!/bin/bash
# Round 5: the parse kernel's instruction mix (one SQ PMC pass) and its floor without the field parse (lib_pfloor).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r05m}
mkdir -p $O
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in base pfloor; do
    if [ $v = base ]; then E="X=1"; else E="GS_LIB_VARIANT=$v"; fi
    env $E timeout -k 10 240 python bench.py --workload ingest --steps 20 --warmup 5 --no-cpu-baseline > $O/ing_${v}_$r.json 2> $O/ing_${v}_$r.err || exit 1
    python -c "import json; d=json.loads(open('$O/ing_${v}_$r.json').read().splitlines()[-1]); r=d['roofline']; print('ingest $v r$r', d['ms_per_step'], r.get('frac'), r.get('frac_wall'), r.get('achieved'))" | tee -a $O/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp
ARGS="--workload ingest --steps 1 --warmup 0 --no-cpu-baseline --no-profile-pass --profile-only"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $O/pmc_sq -o run -- python3 $R/bench.py $ARGS > $O/pmc_sq.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_grbm -o run -- python3 $R/bench.py $ARGS > $O/pmc_grbm.log 2>&1 || exit 1
