"""Summarise a tools/rocprof_round.sh / tools/pmc_workload.sh output directory into
profiles/<tag>_*.{json,md} and, for the workload's dominant kernel, the per-launch
traffic file bench.py reads (profiles/pmc_<workload>_traffic.json; the headline fold's
is profiles/pmc_fold_traffic.json) -- used only when its library hash matches.

Per kernel: dispatches, average duration (kernel trace), and per-dispatch averages of
every PMC counter collected in the separate --pmc passes. Traffic per launch is
L2 -> fabric REQUEST bytes: TCC_EA0_RDREQ x 128 B (+ WRITE_SIZE). On gfx950 FETCH_SIZE
tallies each 128-B request at 64 B (MI355X_MICROARCH.md HBM section: x2), and these
counters count Infinity-Cache hits too -- so the figure is what the L2 asks of the
fabric, an upper bound of HBM bytes, not HBM bytes.
For ingest, the SQ pass gives VALU and LDS activity and LDS bank conflicts.
Usage: python tools/rocprof_summary.py <dir> <tag> <pipeline> [batch] [--workload rmat-cc|rmat20|bip|ingest]
       (<dir> = a summary .json written by an earlier run: only the traffic file is redone)
"""
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict

argv = list(sys.argv[1:])
workload = "rmat-cc"
if "--workload" in argv:
    i = argv.index("--workload")
    workload = argv[i + 1]
    del argv[i:i + 2]
d, tag = argv[0], argv[1]
pipeline = int(argv[2]) if len(argv) > 2 else 3
batch = int(argv[3]) if len(argv) > 3 else 1 << 20
DOMINANT = {"rmat-cc": "k_fold", "rmat20": "k_fold", "bip": "k_fold", "ingest": "k_parse"}[workload]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = {"tag": tag, "pipeline": pipeline, "kernels": {}}


def short(name):
    """'void gs::k_fold<false, true, false>(gs::Table, ...)' -> 'k_fold<false, true, false>'."""
    base = name.replace("void ", "").replace("(anonymous namespace)::", "")
    tmpl = ""
    if "<" in base.split("(")[0]:
        head = base.split("(")[0]
        tmpl = head[head.index("<"):]
        base = head[:head.index("<")]
    else:
        base = base.split("(")[0]
    return base.split("::")[-1] + tmpl


from_summary = d.endswith(".json")
if from_summary:
    with open(d) as f:
        out = json.load(f)
    tr = None
else:
    tr = glob.glob(os.path.join(d, "trace", "*.db"))[0]
    db = sqlite3.connect(tr)
if not from_summary:
    for name, calls, tot, avg, pct in db.execute("select name,total_calls,total_duration,average,percentage from top_kernels"):
        out["kernels"].setdefault(short(name), {}).update(
            {"calls": calls, "total_us": round(tot, 1), "avg_us": round(avg, 3), "pct": round(pct, 2)})

    # busy time of the fold: union of its dispatch intervals in the traced step
    views = [r[0] for r in db.execute("select name from sqlite_master where type in ('view','table')")]
    src = "kernels" if "kernels" in views else [v for v in views if "kernel" in v.lower()][0]
    iv = sorted((s_, e_) for n_, s_, e_ in db.execute("select name, start, end from %s" % src) if DOMINANT in n_)
    busy, cur_s, cur_e = 0, None, None
    for s_, e_ in iv:
        if cur_e is None or s_ > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    if cur_e is not None:
        busy += cur_e - cur_s
    out["%s_busy_ms_per_step" % DOMINANT] = round(busy / 1e6, 3)
    out["%s_span_ms" % DOMINANT] = round((iv[-1][1] - iv[0][0]) / 1e6, 3) if iv else None

    for pdir in sorted(glob.glob(os.path.join(d, "pmc_*"))):
        dbs = glob.glob(os.path.join(pdir, "*.db"))
        if not dbs:
            continue
        c = sqlite3.connect(dbs[0])
        agg = defaultdict(lambda: defaultdict(list))
        for kname, cname, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
            key = short(kname)
            agg[key][cname].append(val)
        for k, cs in agg.items():
            for cname, vals in cs.items():
                out["kernels"].setdefault(k, {})["pmc_" + cname] = round(sum(vals) / len(vals), 3)

    for k in list(out["kernels"]):
        r = out["kernels"][k]
        if "pmc_SQ_WAVE_CYCLES" in r:
            r["derived_sq"] = {
                # VALU instruction-issue cycles per wave-cycle, LDS conflict cycles per LDS-active cycle
                "valu_active_per_wave_cycle": r.get("pmc_SQ_ACTIVE_INST_VALU", 0) / max(r["pmc_SQ_WAVE_CYCLES"], 1),
                "lds_active_per_wave_cycle": r.get("pmc_SQ_ACTIVE_INST_LDS", 0) / max(r["pmc_SQ_WAVE_CYCLES"], 1),
                "lds_bank_conflict_per_lds_active": r.get("pmc_SQ_LDS_BANK_CONFLICT", 0) /
                max(r.get("pmc_SQ_ACTIVE_INST_LDS", 0), 1),
                "valu_insts_per_wave": r.get("pmc_SQ_INSTS_VALU", 0) / max(r.get("pmc_SQ_WAVES", 0), 1),
                "lds_insts_per_wave": r.get("pmc_SQ_INSTS_LDS", 0) / max(r.get("pmc_SQ_WAVES", 0), 1),
            }
            if r.get("pmc_GRBM_GUI_ACTIVE"):  # rocprofv3's derived formulas (rocprofv3 -L, gfx94x fallback), CU_NUM 256
                g = r["pmc_GRBM_GUI_ACTIVE"] * 256.0
                r["derived_sq"]["VALUBusy_pct"] = 100.0 * r.get("pmc_SQ_ACTIVE_INST_VALU", 0) / g
                r["derived_sq"]["LDSBankConflict_pct"] = 100.0 * r.get("pmc_SQ_LDS_BANK_CONFLICT", 0) / g
                if "pmc_SQ_LDS_IDX_ACTIVE" in r:
                    r["derived_sq"]["lds_conflict_per_idx_cycle"] = r.get("pmc_SQ_LDS_BANK_CONFLICT", 0) / max(
                        r["pmc_SQ_LDS_IDX_ACTIVE"] - r.get("pmc_SQ_LDS_BANK_CONFLICT", 0), 1)
        if "pmc_FETCH_SIZE" in r:
            rd_req = r.get("pmc_TCC_EA0_RDREQ_sum")
            r["derived"] = {
                # gfx950: one L2->fabric read request moves 128 B for streaming AND for random
                # 16-B loads (profiles/r01_calib_random_pmc.json); FETCH_SIZE tallies 64 B each.
                "hbm_read_bytes": (rd_req * 128) if rd_req else r["pmc_FETCH_SIZE"] * 1024 * 2,
                "fetch_bytes_raw": r["pmc_FETCH_SIZE"] * 1024,
                "write_bytes": r.get("pmc_WRITE_SIZE", 0) * 1024,
                "read_requests": rd_req,
                "l2_hit_rate": (r["pmc_TCC_HIT_sum"] / (r["pmc_TCC_HIT_sum"] + r["pmc_TCC_MISS_sum"]))
                if "pmc_TCC_HIT_sum" in r else None,
            }
os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
if not from_summary:
    with open(os.path.join(root, "profiles", "%s_rocprof_summary.json" % tag), "w") as f:
        json.dump(out, f, indent=1)
# per-launch traffic of the workload's dominant kernel, read by bench.py (roofline.traffic)
TARGET = {"rmat-cc": ("k_fold<false, false, false>", "rmat26-cc-stream", "pmc_fold_traffic.json"),  # <SIGNED, TRACK, TAKE>
          "rmat20": ("k_fold<false, false, false>", "rmat20-cc-stream", "pmc_r20_traffic.json"),  # config 2
          "bip": ("k_fold<true, false, false>", "bip-config4", "pmc_bip_traffic.json"),
          "ingest": ("k_parse", "ingest-rmat26-text", "pmc_ingest_traffic.json")}[workload]
kname, wname, fname = TARGET
if workload == "ingest" and "k_parse_fused" in out["kernels"]:  # the one-pass parse (round 4 default)
    kname = "k_parse_fused"
if kname not in out["kernels"] and kname.endswith(">") and kname[:-1] + ", false>" in out["kernels"]:
    kname = kname[:-1] + ", false>"  # k_fold<SIGNED, TRACK, TAKE, ROWS> (round 4: the ROWS instantiation)
r = out["kernels"].get(kname, {})
if "derived" in r and r["derived"].get("read_requests"):
    import hashlib
    with open(os.path.join(root, "gelly-streaming_amd", "lib", "libgs_summary.so"), "rb") as f:
        lib_sha16 = hashlib.sha256(f.read()).hexdigest()[:16]
    dv = r["derived"]
    traffic = {
        "round": tag, "workload": wname, "batch": batch, "pipeline": pipeline, "lib_sha16": lib_sha16,
        "kernel": kname, "avg_us_rocprof": r.get("avg_us"), "calls": r.get("calls"),
        "read_requests_per_launch": dv["read_requests"], "bytes_per_read_request": 128,
        "write_bytes_per_launch": dv["write_bytes"],
        "fabric_bytes_per_launch": dv["hbm_read_bytes"] + dv["write_bytes"],
        "fetch_size_kib_raw": r["pmc_FETCH_SIZE"], "l2_hit_rate": dv["l2_hit_rate"],
        "busy_ms_per_step": out.get("%s_busy_ms_per_step" % DOMINANT),
        "traffic_kind": "L2->fabric request bytes (TCC_EA0_RDREQ x 128 B + WRITE_SIZE): Infinity-Cache hits "
                        "included, so an upper bound of HBM bytes",
        "method": "separate rocprofv3 --pmc passes (tools/pmc_workload.sh / tools/rocprof_round.sh, bench defaults: "
                  "pipeline %d) over one bench step; " % pipeline +
                  "read bytes = TCC_EA0_RDREQ x 128 B: on gfx950 one L2->fabric read request moves 128 B both "
                  "for 16-B/lane streaming (256 MiB = 2.10 M requests) and for random 16-B loads (same request "
                  "ceiling), see profiles/r01_calib_random_pmc.json; FETCH_SIZE tallies 64 B per request "
                  "(MI355X_MICROARCH.md HBM section: x2); writes = WRITE_SIZE (KiB)",
        "source": "profiles/%s_rocprof_summary.json" % tag,
    }
    if workload in ("rmat-cc", "rmat20", "bip"):
        traffic["read_requests_per_edge"] = round(dv["read_requests"] / batch, 3)
    if "derived_sq" in r:
        traffic["sq"] = r["derived_sq"]
    if workload == "ingest" and kname == "k_parse":  # the two-pass parse: count pass + parse pass
        cl = out["kernels"].get("k_count_lines", {})
        if "derived" in cl:
            traffic["count_lines"] = {"avg_us_rocprof": cl.get("avg_us"),
                                      "fabric_bytes_per_launch": cl["derived"]["hbm_read_bytes"] +
                                      cl["derived"]["write_bytes"], "sq": cl.get("derived_sq")}
    with open(os.path.join(root, "profiles", fname), "w") as f:
        json.dump(traffic, f, indent=1)
if from_summary:
    sys.exit(0)
lines = ["# rocprofv3 summary %s" % tag, "", "| kernel | calls | avg us | total us | % | extra |", "|---|---|---|---|---|---|"]
for k, r in sorted(out["kernels"].items(), key=lambda kv: -kv[1].get("total_us", 0)):
    extra = ", ".join("%s=%s" % (a[4:], b) for a, b in r.items() if a.startswith("pmc_"))
    if "derived_sq" in r:
        extra += "; " + ", ".join("%s=%.3f" % kv for kv in r["derived_sq"].items())
    lines.append("| %s | %s | %s | %s | %s | %s |" % (k, r.get("calls"), r.get("avg_us"), r.get("total_us"), r.get("pct"), extra))
with open(os.path.join(root, "profiles", "%s_rocprof_summary.md" % tag), "w") as f:
    f.write("\n".join(lines) + "\n")
print("\n".join(lines))
