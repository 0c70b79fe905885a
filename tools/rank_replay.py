"""Per-rank GPU time of the N-GPU exchange path, measured on ONE GPU (diagnostic).

The emulated N-rank run (tools/emulated_scaling.py) shares one GPU between N replicas,
so its time mixes in N tables competing for one chip's caches and N ranks' host work
in one process. This tool instead measures what ONE rank's GPU would do:

  1. record: the exchange protocol of bench.py at N ranks, run rank after rank on one
     GPU through the summary API -- per exchange b, every rank folds its own batch b
     (2^22 edges, first 2^22 per rank every 2^20: the bench's cadence and ramp) with
     delta tracking and takes its records; then folds every other rank's records of
     exchange b - 3 (the native group's lag). Every rank's records are kept;
  2. replay: rank 0 alone -- reset, then per exchange its own tracked fold, the take
     of its records, and the fold of the other ranks' recorded rows of exchange b - 3
     (one launch over all of them, as the native group does),
     all on the summary's stream (no overlap of own and remote folds, which the native
     group has: an upper bound of the rank's GPU time);
  3. compare with the plain 1-GPU pass of the whole stream (T1): projected efficiency
     >= T1 / (N x T_rank). The collectives are not in T_rank: their bytes per rank are
     printed (they overlap the folds on their own streams in the native group).

Also checks rank 0's replica against the single-GPU summary (vertex count and every
label through gs_find_labels_device).

    python tools/rank_replay.py [--scale 26] [--ranks 8] [--reps 3]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lag", type=int, default=3)
    ap.add_argument("--log-batch", type=int, default=22)
    ap.add_argument("--ramp-log2", type=int, default=22)
    ap.add_argument("--ramp-log-batch", type=int, default=20)
    ap.add_argument("--row-stats", action="store_true",
                    help="after the record: rank 0's replay phase by phase (own tracked folds, remote rows), with "
                         "wall time and the debug build's fold counters per phase (GS_LIB_VARIANT=debug for counts)")
    ap.add_argument("--own-only", action="store_true",
                    help="only rank 0's own folds, untracked vs tracked + takes (for a kernel trace of the tax)")
    a = ap.parse_args()
    E, N = 16 << a.scale, a.ranks
    per = E // N
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, a.scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    hint = 1 << (a.scale - 1)  # expected distinct vertices (4 slots each)
    # exchange boundaries of one rank's shard (the ramp, then the cadence)
    bounds, o = [], 0
    while o < per:
        m = (1 << a.ramp_log_batch) if o < (1 << a.ramp_log2) else (1 << a.log_batch)
        m = min(m, per - o)
        bounds.append((o, m))
        o += m
    nex = len(bounds)

    def fold_own(s, r, o, m):
        base = r * per + o
        for x in range(0, m, 1 << 20):
            s.fold_device(src[base + x:], dst[base + x:], n=min(1 << 20, m - x))

    cap = max(m for _, m in bounds) + 256
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    scratch = torch.empty((cap, 3), dtype=torch.int64, device="cuda")
    if a.own_only:
        rep = gs.Summary("cc", capacity_hint=hint)
        for tracked in (False, True, False, True):
            rep.set_delta_tracking(tracked)
            best = None
            for _ in range(a.reps):
                rep.reset()
                rep.sync()
                t = time.perf_counter()
                for o, m in bounds:
                    fold_own(rep, 0, o, m)
                    if tracked:
                        rep.take_delta_records(scratch, cap, cnt)
                rep.sync()
                el = time.perf_counter() - t
                best = el if best is None else min(best, el)
            print("rank 0 own folds %s: %.2f ms" % ("tracked + takes" if tracked else "untracked, no takes",
                                                     best * 1e3), flush=True)
        rep.close()
        return 0

    # 1. record
    summ = [gs.Summary("cc", capacity_hint=hint) for _ in range(N)]
    for s in summ:
        s.set_delta_tracking(True)
    recs = [[None] * nex for _ in range(N)]
    t0 = time.perf_counter()
    for b in range(nex):
        o, m = bounds[b]
        for r in range(N):
            fold_own(summ[r], r, o, m)
            summ[r].take_delta_records(scratch, cap, cnt)
            summ[r].sync()
            k = int(cnt.item())
            recs[r][b] = scratch[:k].clone()
        torch.cuda.current_stream().synchronize()  # the clones (torch's stream) before other summaries fold them
        e = b - a.lag
        if e >= 0:
            for r in range(N):
                for q in range(N):
                    if q != r and recs[q][e].shape[0]:
                        summ[r].fold_records(recs[q][e], recs[q][e].shape[0])
    for e in range(max(0, nex - a.lag), nex):  # the finish: the last data halves
        for r in range(N):
            for q in range(N):
                if q != r and recs[q][e].shape[0]:
                    summ[r].fold_records(recs[q][e], recs[q][e].shape[0])
    for s in summ:
        s.sync()
    t_rec = time.perf_counter() - t0
    sent = [sum(int(x.shape[0]) for x in recs[r]) for r in range(N)]
    nv = [s.num_vertices() for s in summ]
    print("record: %d ranks x %d exchanges in %.1f s; records sent per rank %s (total %d); replica vertices %s"
          % (N, nex, t_rec, sent, sum(sent), nv), flush=True)
    for s in summ[1:]:
        s.close()
    rep0 = summ[0]

    # single-GPU reference: the bench's plain pipelined pass
    one = gs.Summary("cc", capacity_hint=hint)
    one.set_pipelining(3)

    def run_plain():
        one.reset()
        one.sync()
        t = time.perf_counter()
        for x in range(0, E, 1 << 20):
            one.fold_device(src[x:], dst[x:], n=1 << 20)
        one.sync()
        return time.perf_counter() - t

    t1 = min(run_plain() for _ in range(a.reps))
    nv1 = one.num_vertices()
    v = torch.empty(nv1 + 1, dtype=torch.int64, device="cuda")
    lab = torch.empty(nv1 + 1, dtype=torch.int64, device="cuda")
    one.export_labels_device(v, lab)
    v, lab = v[:nv1], lab[:nv1]
    got = torch.empty_like(v)
    fnd = torch.empty(nv1, dtype=torch.uint8, device="cuda")
    rep0.find_labels_device(v, got, fnd)
    rep0.sync()
    exact = nv[0] == nv1 and bool(fnd.all().item()) and bool(torch.equal(got, lab))
    print("single GPU: %.2f ms per pass (%.2f G edges/s); rank 0 replica equals it: %s" % (
        t1 * 1e3, E / t1 / 1e9, exact), flush=True)
    one.close()

    # 2. replay rank 0 alone
    # one launch per exchange over all other ranks' rows, as the native group folds them (one exchange-layout
    # launch on its apply stream), not one small launch per (rank, exchange)
    remote = [[x] if x.shape[0] else [] for x in
              (torch.cat([recs[q][e] for q in range(1, N)]) for e in range(nex))]
    rows = sum(int(x.shape[0]) for e in range(nex) for x in remote[e])
    if a.row_stats:
        row_stats(rep0, bounds, remote, fold_own, scratch, cap, cnt, a.lag, nex, a.reps)

    def run_rank(parts):
        rep0.reset()
        rep0.sync()
        t = time.perf_counter()
        for b in range(nex):
            o, m = bounds[b]
            if "own" in parts:
                fold_own(rep0, 0, o, m)
                if "untracked" not in parts:
                    rep0.take_delta_records(scratch, cap, cnt)
            e = b - a.lag
            if e >= 0 and "remote" in parts:
                for x in remote[e]:
                    rep0.fold_records(x, x.shape[0])
        if "remote" in parts:
            for e in range(max(0, nex - a.lag), nex):
                for x in remote[e]:
                    rep0.fold_records(x, x.shape[0])
        rep0.sync()
        return time.perf_counter() - t

    res = {}
    for parts in (("own",), ("own", "remote")):
        res[parts] = min(run_rank(parts) for _ in range(a.reps))
    t_own, t_all = res[("own",)], res[("own", "remote")]
    # the same own folds untracked and with no takes, serialised (what tracking costs)
    rep0.set_delta_tracking(False)
    t_plain = min(run_rank(("own", "untracked")) for _ in range(a.reps))
    rep0.set_delta_tracking(True)
    print("rank 0 alone: own folds untracked, no takes, serialised %.2f ms" % (t_plain * 1e3), flush=True)
    print("rank 0 alone: own tracked folds + takes %.2f ms; + %d remote rows (%.2f per own edge) %.2f ms" % (
        t_own * 1e3, rows, rows / per, t_all * 1e3), flush=True)
    print("collective bytes per rank per pass: sends %.1f MB, receives %.1f MB (16-B rows)" % (
        sent[0] * 16 / 1e6, rows * 16 / 1e6), flush=True)
    print("projected efficiency at N = %d: T1 / (N x T_rank) = %.2f / (%d x %.2f) = %.3f (ideal T_rank %.2f ms)" % (
        N, t1 * 1e3, N, t_all * 1e3, t1 / (N * t_all), t1 * 1e3 / N), flush=True)
    rep0.close()
    return 0


def row_stats(rep0, bounds, remote, fold_own, scratch, cap, cnt, lag, nex, reps):
    """rank 0's replay, phase by phase: own tracked folds + takes vs the other ranks' rows (serialised,
    synchronised around every phase), with the debug build's fold counters summed per phase."""
    keys = None
    for rep in range(reps):
        rep0.reset()
        rep0.sync()
        tot = {"own": [0.0, None, 0], "remote": [0.0, None, 0]}

        def phase(name, fn, units):
            c0 = rep0.debug_counters()
            rep0.sync()
            t = time.perf_counter()
            fn()
            rep0.sync()
            el = time.perf_counter() - t
            c1 = rep0.debug_counters()
            d = {k: c1[k] - c0[k] for k in c1}
            acc = tot[name]
            acc[0] += el
            acc[1] = d if acc[1] is None else {k: acc[1][k] + d[k] for k in d}
            acc[2] += units

        for b in range(nex):
            o, m = bounds[b]
            phase("own", lambda: (fold_own(rep0, 0, o, m), rep0.take_delta_records(scratch, cap, cnt)), m)
            e = b - lag
            if e >= 0:
                for x in remote[e]:
                    phase("remote", lambda: rep0.fold_records(x, x.shape[0]), int(x.shape[0]))
        for e in range(max(0, nex - lag), nex):
            for x in remote[e]:
                phase("remote", lambda: rep0.fold_records(x, x.shape[0]), int(x.shape[0]))
        for name, (el, d, units) in tot.items():
            per_unit = " ".join("%s %.3f" % (k, d[k] / max(units, 1)) for k in d)
            print("row-stats rep %d %s: %d units in %.2f ms (%.1f G units/s, synchronised per phase); per unit: %s"
                  % (rep, name, units, el * 1e3, units / el / 1e9, per_unit), flush=True)


if __name__ == "__main__":
    sys.exit(main())
