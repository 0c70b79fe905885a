"""Latency-path window modes (diagnostic): per-window host latency p50/p99 of
gs_fold_take_device, one fused launch per window vs the resident window server
(gs_set_window_server), over window sizes 2^6 .. 2^16 edges of the config-5 ER stream
(G(2^22, 2^26), the first `--windows` windows of each size, after a warm-up pass).

    python tools/window_modes.py [--windows 1024]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=1024)
    ap.add_argument("--sizes", default="6,10,12,14,16")
    a = ap.parse_args()
    logn, E = 22, 1 << 26
    s = gs.Summary("cc", device=0, capacity_hint=1 << logn)
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_er(src, dst, 0, E, logn, 0x5EED00E5, True, stream=s.stream)
    s.set_delta_tracking(True)
    cap = (1 << 16) + 16
    rec = torch.empty(cap * 3, dtype=torch.int64, device="cuda")
    cnt = torch.empty(1, dtype=torch.int64, device="cuda")
    s.sync()
    take = gs.lib().gs_fold_take_device
    k = ctypes.c_uint64()
    kr = ctypes.byref(k)
    ps, pd, prec, pcnt = src.data_ptr(), dst.data_ptr(), rec.data_ptr(), cnt.data_ptr()
    for lw in [int(x) for x in a.sizes.split(",")]:
        B = 1 << lw
        n = min(a.windows, E // B)
        row = []
        for mode in ("launch", "server"):
            s.set_window_server(mode == "server")
            best = None
            for _ in range(2):  # warm-up pass, then the measured one
                s.reset()
                lat = np.empty(n)
                for w in range(n):
                    t0 = time.perf_counter()
                    rc = take(s._h, ps + 8 * w * B, pd + 8 * w * B, B, prec, cap, pcnt, kr)
                    lat[w] = time.perf_counter() - t0
                    if rc:
                        raise gs.GSError(rc, gs.lib().gs_last_error().decode())
                best = lat * 1e6
            row.append("%s p50 %.2f p99 %.2f us" % (mode, np.percentile(best, 50), np.percentile(best, 99)))
        print("2^%-2d-edge windows (%d): %s" % (lw, n, "; ".join(row)), flush=True)
    print("server stats: %s" % s.window_server_stats())
    s.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
