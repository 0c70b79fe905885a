#!/bin/bash
# Round 5: one-rank exchange step with the communication streams at the lowest priority (GS_GROUP_LOPRIO=1)
# against normal priority, interleaved, two rounds; the digest check of each line.
set -o pipefail
O=gpurun_out/${1:-r05lp}
mkdir -p $O
for r in 1 2; do for v in normal low; do
  if [ $v = low ]; then E="GS_GROUP_LOPRIO=1"; else E="X=1"; fi
  env $E timeout -k 10 300 python bench.py --exchange --steps 5 --warmup 2 --no-cpu-baseline --no-profile-pass > $O/exch_${v}_$r.json 2> $O/exch_${v}_$r.err || exit 1
  python -c "import json; l=json.loads(open('$O/exch_${v}_$r.json').read().strip().splitlines()[-1]); c=l['config']['self_check']; print('exch $v r$r', l['ms_per_step'], c['digest_equals_single_gpu'], c['replica_label_digests_equal'])" | tee -a $O/summary.txt
done; done
