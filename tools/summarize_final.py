"""Print the key fields of a tools/final_round.sh output directory (one line per bench)."""
import json
import os
import sys

d = sys.argv[1]
for f in ("gpu_tests.out",):
    p = os.path.join(d, f)
    if os.path.exists(p):
        print(open(p).read().strip().splitlines()[-1])
for f in ("bench_n1", "bench_r20", "bench_bip", "bench_er", "bench_ingest", "bench_dropin", "bench_exch"):
    p = os.path.join(d, f + ".out")
    if not os.path.exists(p):
        continue
    lines = [x for x in open(p).read().splitlines() if x.startswith("{")]
    if not lines:
        print(f, "NO LINE")
        continue
    line = json.loads(lines[-1])
    c = line["config"]
    r = line.get("roofline") or {}
    print("== %s value=%s ms=%s frac=%s frac_step=%s fold_us=%s traffic=%s" % (
        f, line["value"], line["ms_per_step"], r.get("frac"), r.get("frac_step"), r.get("fold_avg_us"),
        r.get("traffic")))
    for k in ("self_check", "verdict_parity", "reference_quirk_check", "clean_stream_digest", "p50_us", "p99_us",
              "max_us", "parity", "modes_agree", "tail", "exchange_phases", "odd_cycle_flip_window"):
        if k in c:
            v = c[k]
            if isinstance(v, dict):
                v = {a: b for a, b in v.items() if a != "note"}
            print("   ", k, v)
    for k in ("floor_us", "handoff_floor_us", "request_floor_us", "frac_floor_over_p50", "request_frac_step"):
        if k in r:
            print("   roofline.%s = %s" % (k, r[k]))
