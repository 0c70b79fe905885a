"""Correctness check of the emulated N-rank exchange, pass by pass (diagnostic).

Runs tools/emulated_scaling.py's shape -- N rank threads on one GPU, in-process
communicator (gs_group_set_comm_api: tests/cpp/gs_fake_comm.cpp), summaries reset between passes -- at a scale
the oracle labels in seconds, and compares EVERY replica with the oracle after
EVERY pass. Prints one line per pass and exits 1 on the first difference.

    python tools/emu_check.py [--scale 20] [--ranks 8] [--log-batch 22] [--passes 3]
"""
import argparse
import os
import sys
import threading

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

gs.use_comm_emulation(True)  # in-process collectives (tests/cpp/gs_fake_comm.cpp)
import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--log-batch", type=int, default=22)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--hint-log2", type=int, default=0)
    ap.add_argument("--serial", action="store_true", help="profiling mode: own folds on the handle stream (no lanes)")
    a = ap.parse_args()
    E, B, n = 16 << a.scale, 1 << a.log_batch, a.ranks
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, a.scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    ov, olab = oracle.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    print("oracle: %d vertices" % ov.size, flush=True)
    per = E // n
    uid = gs.group_unique_id()
    summ = [gs.Summary("cc", capacity_hint=1 << (a.hint_log2 or a.scale - 1)) for _ in range(n)]
    if a.serial:
        for s in summ:
            s.set_profiling(True)
    bar = threading.Barrier(n)
    res = [[None] * n for _ in range(a.passes)]
    probe = [None]
    caps = [[None] * n for _ in range(a.passes)]
    errs = []

    def rank(r):
        try:
            g = gs.Group(summ[r], uid, n, r, B)
            for p in range(a.passes):
                summ[r].reset()
                summ[r].sync()
                bar.wait()
                g.fold_batches(src[r * per:], dst[r * per:], per, B)
                g.finish()
                summ[r].sync()
                res[p][r] = summ[r].labels()
                caps[p][r] = (summ[r].table_capacity(), summ[r].capacity_stats())
                if r == 0 and p == a.passes - 1:  # the table itself, looked up id by id
                    probe[0] = summ[r]
                bar.wait()
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
        print("failed: %s" % errs, flush=True)
        return 1
    bad = 0
    for p in range(a.passes):
        for r in range(n):
            v, lab = res[p][r]
            if np.array_equal(v, ov) and np.array_equal(lab, olab):
                continue
            bad += 1
            miss = np.setdiff1d(ov, v).size
            extra = np.setdiff1d(v, ov).size
            same = v.size == ov.size and np.array_equal(v, ov)
            wrong = int((lab != olab).sum()) if same else -1
            print("pass %d rank %d: %d vertices (missing %d, extra %d), wrong labels %d"
                  % (p, r, v.size, miss, extra, wrong), flush=True)
            if miss and r == 0:  # where in the stream the missing vertices occur
                mv = np.setdiff1d(ov, v)
                hs, hd = src.cpu().numpy(), dst.cpu().numpy()
                pos = np.nonzero(np.isin(hs, mv) | np.isin(hd, mv))[0]
                rk, off = pos // per, pos % per
                keys, cnt = np.unique(np.stack([rk, off // B]), axis=1, return_counts=True)
                print("  edges touching them: %d; by (rank, batch): %s" % (pos.size, [
                    (int(a), int(b), int(c)) for (a, b), c in zip(keys.T, cnt)][:24]), flush=True)
                if p == a.passes - 1:  # look the missing ids up in every rank's table
                    keys_t = torch.from_numpy(mv).cuda()
                    lab_t = torch.empty_like(keys_t)
                    fnd = torch.empty(mv.size, dtype=torch.uint8, device="cuda")
                    got = []
                    for q in range(n):
                        summ[q].find_labels_device(keys_t, lab_t, fnd, n=mv.size)
                        summ[q].sync()
                        got.append(int(fnd.sum()))
                    print("  found by lookup, per rank: %s of %d; vertex counts %s" % (
                        got, mv.size, [x.num_vertices() for x in summ]), flush=True)
                for (rq, bq) in set(zip(rk.tolist(), (off // B).tolist())):
                    sel = (rk == rq) & (off // B == bq)
                    blk = np.unique((off[sel] % B) // 256)
                    runs = np.split(blk, np.nonzero(np.diff(blk) != 1)[0] + 1)
                    print("  rank %d batch %d: %d edges in %d of %d blocks, block runs %s" % (
                        rq, bq, int(sel.sum()), blk.size, B // 256,
                        [(int(x[0]), int(x[-1])) for x in runs][:12]), flush=True)
                print("  offsets within the batch: min %d max %d; 2^20 micro-batches %s" % (
                    int((off % B).min()), int((off % B).max()), sorted(set((off % B // (1 << 20)).tolist()))), flush=True)
        print("pass %d done; table capacity / capacity stats per rank: %s" % (p, caps[p]), flush=True)
    for s in summ:
        s.close()
    print("MISMATCHES %d" % bad if bad else "all replicas equal the oracle", flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
