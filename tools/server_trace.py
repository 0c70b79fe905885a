"""Where a resident-server window's latency goes (diagnostic). Runs the config-5 ER stream
(G(2^22, 2^26)) through the window server of the trace build
(make -C gelly-streaming_amd variant V=strace VFLAGS=-DGS_SERVER_TRACE), which stamps
each window's phases with the GPU wall clock (100 MHz), and prints the medians of:

    seen->bcast   block 0: descriptor loaded from the host mailbox and broadcast
    bcast->go     the last block to pick the window up
    go->folded    the slowest block's fold
    folded->done  the publishing block's take_tail (ticket, counts, completion stores)
    device        seen -> completion stored
    host-device   the rest of the host's latency: post -> seen, done -> the host's poll

    GS_LIB_VARIANT=strace python tools/server_trace.py [--windows 1024] [--sizes 6,16]
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
    ap.add_argument("--sizes", default="6,10,16")
    a = ap.parse_args()
    if os.environ.get("GS_LIB_VARIANT") != "strace":
        raise SystemExit("run with GS_LIB_VARIANT=strace (the trace build)")
    L = gs.lib()
    L.gs_debug_server_trace.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
    logn, E = 22, 1 << 26
    s = gs.Summary("cc", device=0, capacity_hint=1 << logn)
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_er(src, dst, 0, E, logn, 0x5EED00E5, True, stream=s.stream)
    s.set_delta_tracking(True)
    cap = (1 << 16) + 16
    rec = torch.empty(cap * 3, dtype=torch.int64, device="cuda")
    cnt = torch.empty(1, dtype=torch.int64, device="cuda")
    TC = 1 << 13
    tr = torch.zeros(TC * 8 + 128, dtype=torch.int64, device="cuda")
    s.sync()
    if L.gs_debug_server_trace(tr.data_ptr(), TC):
        raise SystemExit("gs_debug_server_trace failed")
    take = L.gs_fold_take_device
    k = ctypes.c_uint64()
    kr = ctypes.byref(k)
    ps, pd, prec, pcnt = src.data_ptr(), dst.data_ptr(), rec.data_ptr(), cnt.data_ptr()
    s.set_window_server(True)
    for lw in [int(x) for x in a.sizes.split(",")]:
        B = 1 << lw
        n = min(a.windows, E // B, TC // 2)
        for rep in range(2):  # warm-up pass, then the measured one
            s.reset()  # (stops the server: the next window starts a session)
            tr.zero_()
            torch.cuda.synchronize()
            lat = np.empty(n)
            seqs = []
            for w in range(n):
                t0 = time.perf_counter()
                rc = take(s._h, ps + 8 * w * B, pd + 8 * w * B, B, prec, cap, pcnt, kr)
                lat[w] = time.perf_counter() - t0
                if rc:
                    raise gs.GSError(rc, L.gs_last_error().decode())
            s.sync()  # stops the server: every stamp is in memory
        hist = tr[TC * 8:].cpu().numpy()
        t = tr[:TC * 8].view(TC, 8).cpu().numpy().astype(np.float64)
        t = t[t[:, 5] > 0]  # windows published in the measured pass
        t = t[np.argsort(t[:, 0])][-n:]
        ph = {
            "seen->bcast": (t[:, 1] - t[:, 0]) / 100.0,
            "bcast->go": (t[:, 2] - t[:, 1]) / 100.0,
            "go->folded": (t[:, 3] - t[:, 2]) / 100.0,
            "folded->done": (t[:, 5] - t[:, 4]) / 100.0,
            "device": (t[:, 5] - t[:, 0]) / 100.0,
        }
        host = lat * 1e6
        m = min(len(host), len(t))
        ph["host-device"] = host[-m:] - ph["device"][-m:]
        print("2^%d-edge windows (%d, %d stamped, %d blocks): host p50 %.2f p99 %.2f us" %
              (lw, n, len(t), int(np.median(t[:, 6])), np.percentile(host, 50), np.percentile(host, 99)))
        for kx, v in ph.items():
            print("   %-13s p50 %6.2f  p90 %6.2f us" % (kx, np.percentile(v, 50), np.percentile(v, 90)))
        if len(t) > 128:  # young table (the first 64 windows insert most endpoints) vs the rest
            for nm, sl in (("windows 0-63", slice(0, 64)), ("windows 64-", slice(64, None))):
                print("   %s: host p50 %.2f p99 %.2f | " % (nm, np.percentile(host[-m:][sl], 50),
                                                         np.percentile(host[-m:][sl], 99)) +
                      "  ".join("%s %.2f" % (kx, np.percentile(v[-m:][sl], 50)) for kx, v in ph.items()
                                if kx != "host-device"))
        # per-block fold times over all blocks of the measured pass: old windows, young (first 64) windows
        for nm, hh in (("windows 64-", hist[:64]), ("windows 0-63", hist[64:128])):
            c = np.cumsum(hh)
            if c[-1] == 0:
                continue
            q = lambda f: 0.5 * (int(np.searchsorted(c, f * c[-1])) + 0.5)  # noqa: E731
            print("   per-block fold time, %s (%d blocks): p10 %.2f  p50 %.2f  p90 %.2f  p99 %.2f us" % (
                nm, int(c[-1]), q(0.1), q(0.5), q(0.9), q(0.99)))
        sys.stdout.flush()
    s.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
