"""Per-rank cost of the owner-partitioned N-GPU pass (gs_group_create_partitioned,
DESIGN.md section 5b), measured on ONE GPU.

N rank threads drive N local summaries through the in-process collectives emulation in
SERIALIZED mode (tests/cpp/gs_fake_comm.cpp: a rank holds the GPU token whenever it is
outside a collective), so every rank's work between two collectives runs alone on the GPU
and its HIP events and host clocks time its own work. Per rank and pass:
  own folds (pipelined, untracked in bulk mode; in bulk mode each rank's shard is also folded
  ALONE into a fresh local forest, as a rank's own process would, and that time is the one
  priced) -> combine phases (export + records,
  bucketing, count + row all-to-all (an HBM copy here), owner step, pair all-gather +
  label-forest fold) -> the owned label pass.
The all-to-all is priced from its bytes at a per-link xGMI rate instead of the emulated
copy. The single-GPU pass of the same stream (T1) is timed first and its gs_digest is the
check: the digest of the union of the ranks' owned slices must equal it.

usage: python tools/part_replay.py [--ranks 8] [--scale 26] [--log-edges 30] [--window-log 0]
"""
import argparse
import json
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

SEED = {20: 0x5EED0020, 26: 0x5EED0026}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--log-edges", type=int, default=30)
    ap.add_argument("--window-log", type=int, default=0, help="own edges between combines (0: one per pass)")
    ap.add_argument("--micro-log", type=int, default=20)
    ap.add_argument("--link-gbs", type=float, default=64.0, help="xGMI GB/s per link and direction (model)")
    ap.add_argument("--local-hint", type=int, default=0, help="capacity hint of each rank's local forest (0: V)")
    ap.add_argument("--forest-counters", action="store_true",
                    help="rank 0: the label forest's fold counters after the pass (debug build: GS_LIB_VARIANT=debug)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    N, scale, E = a.ranks, a.scale, 1 << a.log_edges
    per, B = E // N, 1 << a.micro_log
    W = (1 << a.window_log) if a.window_log else 0
    seed = SEED.get(scale, 0x5EED0026)
    V = 1 << (scale - 1)  # expected distinct endpoints (RMAT-26: 32.8 M)
    dev = torch.device("cuda", 0)
    src = torch.empty(E, dtype=torch.int64, device=dev)
    dst = torch.empty(E, dtype=torch.int64, device=dev)
    for o in range(0, E, 1 << 26):
        gs.gen_rmat(src[o:], dst[o:], o, min(1 << 26, E - o), scale, seed, True)
    torch.cuda.synchronize()
    # T1 and the reference digest: the single-GPU pass of bench.py (pipelined 2^20-edge folds)
    with gs.Summary("cc", capacity_hint=V) as s1:
        s1.set_pipelining(3)
        for rep in range(2):
            s1.reset()
            s1.sync()
            t0 = time.perf_counter()
            for o in range(0, E, B):
                s1.fold_device(src[o:], dst[o:], n=min(B, E - o))
            s1.sync()
            t1_ms = (time.perf_counter() - t0) * 1e3
        ref_digest = s1.digest()
        nv_total = s1.num_vertices()
    print("T1 %.2f ms (%d vertices)" % (t1_ms, nv_total), flush=True)
    # each rank's own folds as its own process pays them: its shard into a fresh local forest,
    # pipelined, alone on the GPU (the threaded replay below shares one process's queues and
    # streams between the ranks)
    alone = []
    for r in range(N):
        with gs.Summary("cc", capacity_hint=a.local_hint or V) as sr:
            sr.set_pipelining(3)
            for rep in range(2):
                sr.reset()
                sr.sync()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for o in range(r * per, (r + 1) * per, B):
                    sr.fold_device(src[o:], dst[o:], n=min(B, (r + 1) * per - o))
                sr.sync()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3
            alone.append(ms)
    print("own folds alone per rank (ms):", " ".join("%.2f" % x for x in alone), flush=True)

    gs.use_comm_emulation(True)
    F = gs.fake_comm()
    F.gs_fake_comm_set_serialize(1)
    uid = gs.group_unique_id()
    res = [None] * N
    errs = []

    def rank(r):
        try:
            F.gs_fake_comm_token(1)
            s = gs.Summary("cc", capacity_hint=a.local_hint or V)
            s.set_pipelining(3)
            g = gs.PartGroup(s, uid, N, r, V, W)
            out = {}
            for rep in range(2):  # the second pass is measured
                g.reset()
                s.sync()
                g.set_phase_timing(True)
                fold_ms = fold_dev_ms = fold_nv_ms = 0.0
                lo = r * per
                step = W or per
                torch.cuda.synchronize()  # (device-wide: nothing of another rank's is still running)
                for w0 in range(0, per, step):
                    t0 = time.perf_counter()
                    for o in range(w0, min(per, w0 + step), B):
                        g.fold_device(src[lo + o:], dst[lo + o:], min(B, per - o, w0 + step - o))
                    s.sync()
                    fold_ms += (time.perf_counter() - t0) * 1e3
                    s.num_vertices()  # (a wait through a completion kernel queued behind every lane)
                    fold_nv_ms += (time.perf_counter() - t0) * 1e3
                    torch.cuda.synchronize()  # (a device-wide check that Summary.sync() waited for every lane)
                    fold_dev_ms += (time.perf_counter() - t0) * 1e3
                    g.combine()
                ph = g.phase_stats()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                cap = 4 * (V // N) + (1 << 20)
                ov = torch.empty(cap, dtype=torch.int64, device=dev)
                ol = torch.empty(cap, dtype=torch.int64, device=dev)
                k = g.labels_device(ov, ol)
                labels_ms = (time.perf_counter() - t0) * 1e3
                st = g.stats()
                if a.forest_counters and r == 0:
                    print("label forest counters (rank 0):", g.forest_counters(), flush=True)
                out = {"rank": r, "own_fold_ms": fold_ms, "own_fold_device_sync_ms": fold_dev_ms, "own_fold_nv_ms": fold_nv_ms, "labels_ms": labels_ms, **ph, **st, "owned": k}
                out["digest"] = gs.digest_rows(ov[:k], ol[:k])
                del ov, ol
            g.close()
            s.close()
            res[r] = out
        except BaseException as e:  # noqa: BLE001
            errs.append((r, repr(e)))
        finally:
            F.gs_fake_comm_token(0)

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    F.gs_fake_comm_set_serialize(0)
    gs.use_comm_emulation(False)
    if errs:
        print("errors", errs)
        sys.exit(1)
    digest = sum(x["digest"] for x in res) & ((1 << 64) - 1)
    width_b = 16
    rows = []
    max_pairs = max(x["pairs_sent"] for x in res)
    for x in res:
        # the collectives priced at the link rate (the emulation's phases [3], [5] wait for the
        # other ranks): this rank's rows to the N-1 other owners, one link each, and the pair
        # all-gather (every rank sends its max-count-padded pairs to every other rank)
        sent_b = x["rows_exported"] * width_b
        a2a_model = (sent_b / max(N, 1)) / (a.link_gbs * 1e9) * 1e3 if N > 1 else 0.0
        gather_model = (max_pairs * width_b) / (a.link_gbs * 1e9) * 1e3 if N > 1 else 0.0
        comp = x["export_ms"] + x["bucket_ms"] + x["owner_ms"] + x["forest_fold_ms"]
        x["a2a_model_ms"] = a2a_model
        x["pair_gather_model_ms"] = gather_model
        x["combine_compute_ms"] = comp
        x["own_fold_alone_ms"] = alone[x["rank"]]
        # (windowed: the own folds are tracked, timed in the threaded run to a device-wide sync)
        own = x["own_fold_alone_ms"] if W == 0 else x["own_fold_device_sync_ms"]
        x["rank_ms"] = own + comp + a2a_model + gather_model + x["labels_ms"]
        rows.append(x)
    tmax = max(x["rank_ms"] for x in rows)
    summary = {
        "ranks": N, "scale": scale, "edges": E, "window": W, "T1_ms": t1_ms, "vertices": nv_total,
        "digest_equal": digest == ref_digest, "rank_ms_max": tmax,
        "efficiency_projected": t1_ms / (N * tmax),
        "sum_rows_exported_over_V": sum(x["rows_exported"] for x in rows) / nv_total,
        "pairs_folded_over_V": rows[0]["pairs_folded"] / nv_total,
        "label_forest_vertices_over_V": rows[0]["label_forest_vertices"] / nv_total,
        "per_rank": rows,
    }
    print(json.dumps(summary, indent=1), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)
    sys.exit(0 if summary["digest_equal"] else 2)


if __name__ == "__main__":
    main()
