set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
for v in plbs plbsfl; do
  GS_LIB_VARIANT=$v timeout -k 10 240 python bench.py --workload ingest --steps 5 --warmup 2 --no-cpu-baseline > $O/$v.json 2> $O/$v.err || exit 1
  grep -E "LBSTATS|LBPHASES" $O/$v.err > $O/$v.lbs.txt
done
