"""Work inflation of the N-rank exchange path, measured on ONE GPU.

N rank threads each drive their own replica through the native group
(include/gs_group.h) with the in-process communicator emulation
(gs_group_set_comm_api: tests/cpp/gs_fake_comm.cpp): every rank folds its contiguous 1/N shard of the RMAT
stream in per-rank micro-batches, stages its structural delta, "all-gathers" it
(device copies) and folds the other ranks' rows -- exactly bench.py's N-GPU step,
with all N ranks' work sharing one GPU. With perfect scaling the N ranks' total
work equals the 1-rank pass without exchange, so

    inflation(N) = T_emulated(N) / T_plain(1)

bounds the N-GPU efficiency from above by 1 / inflation(N) (the xGMI transfer is
replaced by an HBM copy; launch concurrency across ranks is what one GPU allows).

    python tools/emulated_scaling.py [--scale 26] [--ranks 1,2,4,8] [--reps 2]
"""
import argparse
import os
import sys
import threading
import time

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402

gs.use_comm_emulation(True)  # in-process collectives (tests/cpp/gs_fake_comm.cpp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=26)
    ap.add_argument("--log-batch", type=int, default=22, help="edges per rank between exchanges (log2)")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--hint-log2", type=int, default=0, help="capacity hint of the rank replicas (0: 2^scale)")
    ap.add_argument("--ramp-log2", type=int, default=22,
                    help="first 2^ramp-log2 edges per rank exchanged every --ramp-log-batch edges "
                         "(gs_group_set_ramp; 0: no ramp)")
    ap.add_argument("--ramp-log-batch", type=int, default=20)
    a = ap.parse_args()
    E, B = 16 << a.scale, 1 << a.log_batch
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, a.scale, 0x5EED0026, True)
    torch.cuda.synchronize()

    # baseline: one summary, no exchange, pipelined folds (bench.py at N = 1)
    s = gs.Summary("cc", capacity_hint=1 << (a.scale - 1))
    s.set_pipelining(3)
    best = 1e9
    for _ in range(a.reps + 1):
        s.reset()
        t0 = time.perf_counter()
        for o in range(0, E, B):
            s.fold_device(src[o:], dst[o:], n=min(B, E - o))
        s.sync()
        best = min(best, time.perf_counter() - t0)
    s.close()
    t1 = best
    print("plain 1 rank: %.2f ms" % (t1 * 1e3), flush=True)

    for n in [int(x) for x in a.ranks.split(",")]:
        per = E // n
        uid = gs.group_unique_id()
        summ = [gs.Summary("cc", capacity_hint=1 << (a.hint_log2 or a.scale - 1)) for _ in range(n)]
        bar = threading.Barrier(n)
        times = [[] for _ in range(n)]
        recs = [None] * n
        errs = []

        def rank(r):
            try:
                g = gs.Group(summ[r], uid, n, r, B)
                g.set_ramp(1 << a.ramp_log2 if a.ramp_log2 else 0, 1 << a.ramp_log_batch)
                for _ in range(a.reps + 1):
                    summ[r].reset()
                    summ[r].sync()
                    bar.wait()
                    t0 = time.perf_counter()
                    g.fold_batches(src[r * per:], dst[r * per:], per, B)
                    g.finish()
                    summ[r].sync()
                    times[r].append(time.perf_counter() - t0)
                    bar.wait()
                recs[r] = g.stats()
                g.close()
            except BaseException as e:  # noqa: BLE001
                errs.append((r, repr(e)))
                bar.abort()

        ts = [threading.Thread(target=rank, args=(r,)) for r in range(n)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            print("N=%d failed: %s" % (n, errs), flush=True)
            return 1
        nv = [x.num_vertices() for x in summ]
        for x in summ:
            x.close()
        tn = min(max(times[r][k] for r in range(n)) for k in range(1, a.reps + 1))
        sent = sum(x["records_sent"] for x in recs)
        print("N=%d: %.2f ms for all ranks on one GPU, inflation %.2fx (efficiency bound %.2f); "
              "exchanges/rank %d (all passes), records sent by all ranks in the last pass %d, rows received by rank 0 per pass %d; "
              "vertices %s"
              % (n, tn * 1e3, tn / t1, t1 / tn, recs[0]["exchanges"], sent,
                 recs[0]["rows_received"] // (a.reps + 1), sorted(set(nv))), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
