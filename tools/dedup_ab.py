"""A/B of micro-batch dedup by hashing (gs_set_batch_dedup) on one GPU (diagnostic).

Pass time with the dedup pre-pass off and on, pipelined as bench.py folds (depth 3):
  rmat26    config 3: RMAT-26, 2^30 edges, 2^20-edge batches (repeats are rare)
  rmat20    config 2: RMAT-20, 2^24 edges, 2^20-edge batches
  rep10     a repeat-heavy stream shaped like the reference's bipartite example
            (BipartitenessCheckExample.java:109-118: every edge 10 times in a row):
            2^20 RMAT-20 edges, each written 10 times, 2^20-edge batches
  rep10w16  the same stream in 2^16-edge windows (the table stays L2-resident)
Labels are compared between the two modes (device lookups of every vertex).

    python tools/dedup_ab.py [--reps 3]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def run(src, dst, B, hint, dedup, reps, depth=3):
    s = gs.Summary("cc", capacity_hint=hint)
    s.set_pipelining(depth)
    s.set_batch_dedup(dedup)
    best = 1e9
    E = src.numel()
    for _ in range(reps + 1):
        s.reset()
        s.sync()
        t0 = time.perf_counter()
        for o in range(0, E, B):
            s.fold_device(src[o:], dst[o:], n=min(B, E - o))
        s.sync()
        best = min(best, time.perf_counter() - t0)
    return s, best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="")
    ap.add_argument("--pipeline", type=int, default=3)
    ap.add_argument("--off-only", action="store_true", help="time the plain fold only")
    a = ap.parse_args()
    cases = []
    for name, scale, n, B, rep in (("rmat26", 26, 1 << 30, 1 << 20, 1), ("rmat20", 20, 1 << 24, 1 << 20, 1),
                                    ("rep10", 20, 1 << 20, 1 << 20, 10), ("rep10w16", 20, 1 << 20, 1 << 16, 10)):
        if a.only and name not in a.only.split(","):
            continue
        cases.append((name, scale, n, B, rep))
    for name, scale, n, B, rep in cases:
        src = torch.empty(n, dtype=torch.int64, device="cuda")
        dst = torch.empty(n, dtype=torch.int64, device="cuda")
        gs.gen_rmat(src, dst, 0, n, scale, 0x5EED0026, True)
        if rep > 1:
            src = src.repeat_interleave(rep)
            dst = dst.repeat_interleave(rep)
        torch.cuda.synchronize()
        hint = 1 << scale
        s0, t0 = run(src, dst, B, hint, False, a.reps, a.pipeline)
        if a.off_only:
            print("%-9s pipeline %d: plain %.3f ms" % (name, a.pipeline, t0 * 1e3), flush=True)
            s0.close()
            continue
        s1, t1 = run(src, dst, B, hint, True, a.reps, a.pipeline)
        nv = s0.num_vertices()
        v = torch.empty(nv + 1, dtype=torch.int64, device="cuda")
        lab = torch.empty(nv + 1, dtype=torch.int64, device="cuda")
        s0.export_labels_device(v, lab)
        got = torch.empty(nv, dtype=torch.int64, device="cuda")
        fnd = torch.empty(nv, dtype=torch.uint8, device="cuda")
        s1.find_labels_device(v[:nv], got, fnd)
        s1.sync()
        same = s1.num_vertices() == nv and bool(fnd.all().item()) and bool(torch.equal(got, lab[:nv]))
        E = src.numel()
        print("%-9s %d edges, %d-edge batches: dedup off %.3f ms (%.2f G edges/s), on %.3f ms (%.2f G edges/s), "
              "on/off %.2f; summaries equal: %s" % (name, E, B, t0 * 1e3, E / t0 / 1e9, t1 * 1e3, E / t1 / 1e9,
                                                   t1 / t0, same), flush=True)
        s0.close()
        s1.close()
        del src, dst, v, lab, got, fnd
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
