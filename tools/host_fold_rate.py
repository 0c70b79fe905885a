"""PCIe-inclusive rate of the drop-in boundary (SURVEY.md 8(d) "secondary" figure):
gs_fold from HOST memory (the call a JVM summary makes when it flushes), RMAT-26
edges in 2^20-edge micro-batches, from pageable numpy arrays and from pinned
(page-locked) torch tensors. gs_fold has HIP copy each 2^20-edge chunk straight
from the caller's buffer into device staging and folds it there; the timing
includes the H2D transfer and the fold (synchronised at the end). Never bench.py's
value.

    python tools/host_fold_rate.py [--log-edges 26]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-edges", type=int, default=26)
    a = ap.parse_args()
    E, B = 1 << a.log_edges, 1 << 20
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, 26, 0x5EED0026, True)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()                 # pageable
    ps, pd = src.cpu().pin_memory(), dst.cpu().pin_memory()       # pinned
    del src, dst
    s = gs.Summary("cc", capacity_hint=1 << 25)
    L = gs.lib()
    for name, xs, xd in (("pageable", hs.ctypes.data, hd.ctypes.data), ("pinned", ps.data_ptr(), pd.data_ptr())):
        best = 1e9
        for _ in range(3):
            s.reset()
            s.sync()
            t0 = time.perf_counter()
            for o in range(0, E, B):
                rc = L.gs_fold(s._h, xs + 8 * o, xd + 8 * o, B)
                if rc:
                    raise gs.GSError(rc, L.gs_last_error().decode())
            s.sync()
            best = min(best, time.perf_counter() - t0)
        print("%-8s host edges: %.1f ms for 2^%d edges = %.2f G edges/s (%.1f GB/s of edges)"
              % (name, best * 1e3, a.log_edges, E / best / 1e9, 16 * E / best / 1e9), flush=True)
    s.close()


if __name__ == "__main__":
    main()
