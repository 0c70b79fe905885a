"""Diagnostic: the first micro-batches of a fresh summary cost 4-6x a steady-state one
(RMAT-20: 150 vs 28 us; bipartite config 4: 166 / 88 / 53 vs 42 us). Time the first
two 2^20-edge batches folded as 2^20 / k-edge launches (k = 1..16), serialised on the
handle stream, for the CC RMAT-20 stream (config 2) and the signed bipartite stream
(config 4); labels are checked against a reference run.
    python tools/first_batch_split.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 1 << 20
    E = 4 * B
    cases = []
    s = torch.empty(E, dtype=torch.int64, device=dev)
    d = torch.empty(E, dtype=torch.int64, device=dev)
    gs.gen_rmat(s, d, 0, E, 20, 0x5EED0020, True)
    cases.append(("cc", "rmat20", s, d, 1 << 20))
    s2 = torch.empty(E, dtype=torch.int64, device=dev)
    d2 = torch.empty(E, dtype=torch.int64, device=dev)
    gs.gen_bip(s2, d2, 0, E, 19, 0x5EED0B1B, [])
    cases.append(("signed", "bip", s2, d2, 1 << 20))
    torch.cuda.synchronize()
    for kind, name, src, dst, hint in cases:
        summ = gs.Summary(kind, capacity_hint=hint)
        ref = None
        for k in (1, 2, 4, 8, 16, 1, 4):
            best = None
            for rep in range(3):
                summ.reset()
                summ.sync()
                t0 = time.perf_counter()
                for b in range(2):  # batches 0 and 1
                    step = B // k
                    for o in range(b * B, (b + 1) * B, step):
                        summ.fold_device(src[o:], dst[o:], n=step)
                summ.sync()
                el = (time.perf_counter() - t0) * 1e6
                best = el if best is None else min(best, el)
            for o in range(2 * B, E, B):  # the rest, for the label check
                summ.fold_device(src[o:], dst[o:], n=B)
            v, lab = summ.labels()
            if ref is None:
                ref = (v, lab)
            ok = np.array_equal(ref[0], v) and np.array_equal(ref[1], lab)
            print("%-7s batches 0+1 as %2d launches each: %7.1f us  (labels %s)" % (name, k, best, "ok" if ok else "DIFFER"),
                  flush=True)
        summ.close()


if __name__ == "__main__":
    main()
