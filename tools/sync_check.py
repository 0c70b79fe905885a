"""Own-fold time of one rank's shard in a fresh process (what a rank of an N-GPU run pays):
128 x 2^20-edge pipelined folds of a 2^27-edge RMAT-26 segment, closed by Summary.sync() or by a
device-wide synchronisation -- a plain summary at two stream offsets, and the local forest of a
one-rank partitioned group (collectives emulated) with its lanes created before or after the
group's label forest (the streams' order decides which hardware queues the lanes land on)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

E, B = 1 << 27, 1 << 20


def folds(s, src, dst, g=None, how="sync"):
    if g is not None:
        g.reset()
    else:
        s.reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for o in range(0, E, B):
        if g is not None:
            g.fold_device(src[o:], dst[o:], B)
        else:
            s.fold_device(src[o:], dst[o:], n=B)
    if how == "device":
        torch.cuda.synchronize()
    else:
        s.sync()
    return (time.perf_counter() - t0) * 1e3


def main():
    src = torch.empty(2 * E, dtype=torch.int64, device="cuda")
    dst = torch.empty(2 * E, dtype=torch.int64, device="cuda")
    for o in range(0, 2 * E, 1 << 26):
        gs.gen_rmat(src[o:], dst[o:], o, 1 << 26, 26, 0x5EED0026, True)
    torch.cuda.synchronize()
    for off in (0, E):
        with gs.Summary("cc", capacity_hint=1 << 25) as s:
            s.set_pipelining(3)
            t = [folds(s, src[off:], dst[off:], how=h) for h in ("sync", "device", "sync", "device")]
            print("plain summary, offset %10d: %s ms" % (off, " ".join("%.2f" % x for x in t)), flush=True)
    gs.use_comm_emulation(True)
    for lanes_first in (True, False):
        with gs.Summary("cc", capacity_hint=1 << 25) as s:
            if lanes_first:
                s.set_pipelining(3)
            g = gs.PartGroup(s, gs.group_unique_id(), 1, 0, 1 << 25, 0)
            if not lanes_first:
                s.set_pipelining(3)
            t = []
            for h in ("sync", "device", "sync", "device"):
                t.append(folds(s, src, dst, g, h))
                g.combine()
            print("partitioned local forest, lanes %s the label forest: %s ms" % (
                "before" if lanes_first else "after", " ".join("%.2f" % x for x in t)), flush=True)
            g.close()
    gs.use_comm_emulation(False)


if __name__ == "__main__":
    main()
