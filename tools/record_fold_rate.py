"""Cost of folding exchange records vs folding edges, on one GPU (diagnostic).

At N GPUs every rank folds its own 1/N of the edges plus the other ranks' hook
records. This measures, on RMAT-26 shards as bench.py cuts
them at N = 8:
  edges     fold rank 0's shard (2^27 edges) into a fresh summary;
  records   rank 0's shard folded with delta tracking, its records taken every
            2^22 edges; then those records folded into
              (a) a fresh summary,
              (b) a summary holding rank 1's shard (what a receiving rank holds),
              (c) the summary that produced them (every row already joined).

    python tools/record_fold_rate.py [--scale 26] [--ranks 8]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def timed(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        t = fn()
        best = min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--ranks", type=int, default=8)
    a = ap.parse_args()
    E = 16 << a.scale
    per = E // a.ranks
    B = 1 << 22
    src = torch.empty(2 * per, dtype=torch.int64, device="cuda")
    dst = torch.empty(2 * per, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, 2 * per, a.scale, 0x5EED0026, True)  # ranks 0 and 1's shards
    torch.cuda.synchronize()
    hint = 1 << a.scale

    def fold_edges(s, o, n):
        for x in range(o, o + n, 1 << 20):
            s.fold_device(src[x:], dst[x:], n=min(1 << 20, o + n - x))

    # records of rank 0's shard, taken every 2^22 edges (the exchange cadence)
    prod = gs.Summary("cc", capacity_hint=hint)
    prod.set_delta_tracking(True)
    cap = prod.delta_capacity()
    rec = torch.empty((per, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    nrec = 0
    for o in range(0, per, B):
        fold_edges(prod, o, min(B, per - o))
        prod.take_delta_records(rec[nrec:], min(cap, per - nrec), cnt)
        prod.sync()
        nrec += int(cnt.item())
    print("rank 0 shard: %d edges -> %d records (%.3f per edge)" % (per, nrec, nrec / per), flush=True)

    s = gs.Summary("cc", capacity_hint=hint)
    s.set_pipelining(3)

    def run_edges():
        s.reset()
        s.sync()
        t0 = time.perf_counter()
        fold_edges(s, 0, per)
        s.sync()
        return time.perf_counter() - t0

    te = timed(run_edges)

    def run_records(pre):
        s.reset()
        if pre is not None:
            fold_edges(s, pre, per)
        s.sync()
        t0 = time.perf_counter()
        s.fold_records(rec, nrec)
        s.sync()
        return time.perf_counter() - t0

    # the same shard as a group's tracked own folds (1 rank, in-process communicator: 3 fold
    # lanes, per-exchange stage + count/data collectives, no remote rows) vs the plain fold
    gs.use_comm_emulation(True)
    g = gs.Group(s, gs.group_unique_id(), 1, 0, B)

    def run_tracked():
        s.reset()
        s.sync()
        t0 = time.perf_counter()
        g.fold_batches(src, dst, per, B)
        g.finish()
        s.sync()
        return time.perf_counter() - t0

    tt = timed(run_tracked)
    g.close()
    print("tracked own fold (1-rank group, exchange every 2^22): %.2f ms (%.2f G edges/s, %.3f x the plain fold)"
          % (tt * 1e3, per / tt / 1e9, tt / te), flush=True)
    s.set_pipelining(3)
    ta = timed(lambda: run_records(None))
    tb = timed(lambda: run_records(per))
    tc = timed(lambda: run_records(0))
    print("edges: %.2f ms (%.2f G edges/s)" % (te * 1e3, per / te / 1e9))
    for name, t in (("records into a fresh summary", ta), ("records into rank 1's replica", tb),
                    ("records into their producer (all joined)", tc)):
        print("%s: %.2f ms (%.2f G rows/s, %.2f x the per-edge cost)" % (name, t * 1e3, nrec / t / 1e9,
                                                                        (t / nrec) / (te / per)), flush=True)
    s.close()
    prod.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
