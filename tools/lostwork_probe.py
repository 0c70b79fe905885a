"""Lost-work probe: one instrumented run of the emulated N-rank
exchange with the conditions under which round 2 lost whole-XCD shares of own folds
(highest-priority comm streams, many hardware queues), using the block-log build
(make -C gelly-streaming_amd blocklog): every CC k_fold workgroup appends
{start/end clock, src, table, blockIdx, gridDim, n, XCC_ID, HW_ID, valid edges, fresh
inserts, hook attempts}. After every pass each replica's vertex count is compared
with the oracle's; on a mismatch the log answers, for every own-fold block whose
edges name a missing vertex: was it dispatched at all, with which arguments, on which
XCD, and what did its edges find.

    make -C gelly-streaming_amd blocklog BLFLAGS=-DGS_GROUP_HIPRIO=1
    GPU_MAX_HW_QUEUES=32 GS_LIB_VARIANT=blocklog python tools/lostwork_probe.py --ranks 8 --passes 4
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

LOG_DT = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("src", "<u8"), ("tab", "<u8"), ("blk", "<u4"), ("nblk", "<u4"),
                   ("n", "<u4"), ("xcc", "<u4"), ("hwid", "<u4"), ("valid", "<u4"), ("fresh", "<u4"),
                   ("hooks", "<u4")])
MICRO = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=20)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--log-batch", type=int, default=22)
    ap.add_argument("--passes", type=int, default=4)
    ap.add_argument("--log-cap", type=int, default=1 << 22)
    a = ap.parse_args()
    L = gs.lib()
    if not hasattr(L, "gs_debug_blocklog"):
        raise SystemExit("needs the block-log build: make -C gelly-streaming_amd blocklog; GS_LIB_VARIANT=blocklog")
    import ctypes
    L.gs_debug_blocklog.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
    L.gs_debug_blocklog_count.restype = ctypes.c_ulonglong
    print("env: GPU_MAX_HW_QUEUES=%s" % os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
    E, B, n = 16 << a.scale, 1 << a.log_batch, a.ranks
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, a.scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    ov, olab = oracle.cc_labels(hs, hd)
    print("oracle: %d vertices" % ov.size, flush=True)
    per = E // n
    base = src.data_ptr()
    log = torch.zeros(a.log_cap * LOG_DT.itemsize, dtype=torch.uint8, device="cuda")
    uid = gs.group_unique_id()
    summ = [gs.Summary("cc", capacity_hint=1 << a.scale) for _ in range(n)]
    tabs = {}
    bar = threading.Barrier(n)
    errs = []
    counts = [None] * n
    stop = [False]

    def rank(r, p, g):
        try:
            summ[r].reset()
            summ[r].sync()
            bar.wait()
            g.fold_batches(src[r * per:], dst[r * per:], per, B)
            g.finish()
            summ[r].sync()
            counts[r] = summ[r].num_vertices()
            bar.wait()
        except BaseException as e:  # noqa: BLE001
            errs.append((r, repr(e)))
            bar.abort()

    groups = [None] * n

    def make(r):
        groups[r] = gs.Group(summ[r], uid, n, r, B)

    ts = [threading.Thread(target=make, args=(r,)) for r in range(n)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    bad_pass = None
    for p in range(a.passes):
        torch.cuda.synchronize()
        assert L.gs_debug_blocklog(log.data_ptr(), a.log_cap) == 0
        ts = [threading.Thread(target=rank, args=(r, p, groups[r])) for r in range(n)]
        [t.start() for t in ts]
        [t.join() for t in ts]
        if errs:
            print("failed: %s" % errs, flush=True)
            return 2
        nlog = int(L.gs_debug_blocklog_count())
        ok = all(c == ov.size for c in counts)
        print("pass %d: vertex counts %s (oracle %d), %d block records%s" % (
            p, counts, ov.size, nlog, "" if ok else "  <-- MISMATCH"), flush=True)
        rec = np.frombuffer(log[:min(nlog, a.log_cap) * LOG_DT.itemsize].cpu().numpy().tobytes(), dtype=LOG_DT)
        # own-fold launches: src inside the edge array
        own = rec[(rec["src"] >= base) & (rec["src"] < base + 8 * E)]
        launches = {}
        for x in own:
            launches.setdefault((int(x["src"]), int(x["tab"])), []).append(x)
        short = [(k, len(v), int(v[0]["nblk"])) for k, v in launches.items() if len(v) != int(v[0]["nblk"])]
        xccs = np.bincount(own["xcc"] & 15, minlength=8)
        print("  own-fold launches %d, with missing workgroups %d; workgroups per XCC_ID %s" % (
            len(launches), len(short), xccs.tolist()), flush=True)
        for (s_, t_), got, want in short[:16]:
            v = launches[(s_, t_)]
            blks = np.array(sorted(int(x["blk"]) for x in v))
            missing = np.setdiff1d(np.arange(want), blks)
            print("    launch src+%d tab %#x: %d of %d workgroups logged; missing blk mod 8 %s; XCC of logged %s" % (
                (s_ - base) // 8, t_, got, want, np.unique(missing % 8).tolist(),
                np.unique([int(x["xcc"]) & 15 for x in v]).tolist()), flush=True)
        if not ok:
            bad_pass = p
            for r in range(n):
                tabs[r] = None
            v, lab = summ[0].labels()
            mv = np.setdiff1d(ov, v)
            print("  rank 0 misses %d vertices" % mv.size, flush=True)
            pos = np.nonzero(np.isin(hs, mv) | np.isin(hd, mv))[0]
            seen = set()
            for q_pos in pos[:4096]:
                q, off = int(q_pos // per), int(q_pos % per)
                lsrc = base + 8 * (q * per + (off - off % MICRO))
                blk = (off % MICRO) // 256
                if (lsrc, blk) in seen:
                    continue
                seen.add((lsrc, blk))
                m = own[(own["src"] == lsrc) & (own["blk"] == blk)]
                if m.size == 0:
                    print("    edge %d (rank %d, off %d): block %d of launch src+%d NEVER LOGGED" % (
                        q_pos, q, off, blk, (lsrc - base) // 8), flush=True)
                else:
                    for x in m:
                        print("    edge %d (rank %d, off %d): block %d ran on XCC %d (hwid %#x), n %d, valid %d, "
                              "fresh %d, hooks %d, tab %#x, %.1f us" % (
                                  q_pos, q, off, blk, int(x["xcc"]) & 15, int(x["hwid"]), int(x["n"]),
                                  int(x["valid"]), int(x["fresh"]), int(x["hooks"]), int(x["tab"]),
                                  (int(x["t1"]) - int(x["t0"])) / 100.0), flush=True)
                if len(seen) >= 24:
                    break
            break
    for g in groups:
        g.close()
    for s in summ:
        s.close()
    print("RESULT: %s" % ("lost work reproduced in pass %d" % bad_pass if bad_pass is not None
                          else "every replica exact in every pass"), flush=True)
    return 1 if bad_pass is not None else 0


if __name__ == "__main__":
    sys.exit(main())
