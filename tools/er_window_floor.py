"""Config-5 window anatomy (diagnostic): k_fold duration (HIP events, serialised) of one
2^16-edge ER window in steady state, for
  fresh     the window's first fold (hooks of that window included)
  refold    the same window again (every edge already joined: edge load + probes +
            shortcut/find only) -- the floor of a 2^16-edge launch
  tiny      a 64-edge launch of the same kind (launch + one dependent chain)
    python tools/er_window_floor.py [--at 512]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--at", type=int, default=512)
    ap.add_argument("--track", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    logn, E, B = 22, 1 << 26, 1 << 16
    s = gs.Summary("cc", device=0, capacity_hint=1 << logn)
    src = torch.empty(E, dtype=torch.int64, device=dev)
    dst = torch.empty(E, dtype=torch.int64, device=dev)
    gs.gen_er(src, dst, 0, E, logn, 0x5EED00E5, True, stream=s.stream)
    cap = 3 * B + 16
    rec = torch.empty(cap * 3, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    ps, pd = src.data_ptr(), dst.data_ptr()
    res = {}
    for w in range(a.at, a.at + 16):
        s.set_delta_tracking(False)
        s.reset()
        for o in range(0, w * B, 1 << 20):
            s.fold_device(ps + 8 * o, pd + 8 * o, n=min(1 << 20, w * B - o))
        s.set_delta_tracking(bool(a.track))
        s.sync()
        s.set_profiling(True)
        o = w * B
        for kind in ("fresh", "refold", "refold", "tiny"):
            n = 64 if kind == "tiny" else B
            s.fold_device(ps + 8 * o, pd + 8 * o, n=n)
            s.sync()
            k, ms = s.kernel_stats("fold")
            res.setdefault(kind, []).append(ms * 1e3 / max(k, 1))
            s.set_profiling(False)
            s.set_profiling(True)
            if a.track:
                s.take_delta_records(rec, cap, cnt)
        s.set_profiling(False)
    for k, v in res.items():
        v = np.array(v)
        print("%-7s k_fold p50 %6.2f us  min %6.2f  max %6.2f" % (k, np.median(v), v.min(), v.max()), flush=True)
    s.close()


if __name__ == "__main__":
    main()
