"""Where the config-5 per-window latency goes (diagnostic). ER G(2^22, 2^26), 2^16-edge
windows, delta tracking on; p50 / p99 microseconds per window for:
  separate   torch slices, fold_device, take_delta_records, gs_sync (three launches)
  rawptr     the same with precomputed integer device pointers (no torch slicing)
  fold_sync  rawptr without the delta take
  fused      gs_fold_take_device (one launch: fold + take + completion word)
  sync_only  an empty gs_sync per window (host <-> device round trip)
    python tools/er_latency_probe.py
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
    logn, E, B = 22, 1 << 26, 1 << 16
    s = gs.Summary("cc", device=0, capacity_hint=1 << logn)
    src = torch.empty(E, dtype=torch.int64, device=dev)
    dst = torch.empty(E, dtype=torch.int64, device=dev)
    gs.gen_er(src, dst, 0, E, logn, 0x5EED00E5, True, stream=s.stream)
    s.set_delta_tracking(True)
    cap = 3 * B + 16
    rec = torch.empty(cap * 3, dtype=torch.int64, device=dev)
    cnt = torch.empty(1, dtype=torch.int64, device=dev)
    s.sync()
    L = gs.lib()
    s2 = gs.Summary("cc", device=0, capacity_hint=1 << logn)  # fold_sync: no delta tracking
    ps, pd, pr, pc = src.data_ptr(), dst.data_ptr(), rec.data_ptr(), cnt.data_ptr()

    def check(rc):
        if rc:
            raise gs.GSError(rc, L.gs_last_error().decode())

    def run(kind):
        x = s2 if kind == "fold_sync" else s
        x.reset()
        x.sync()
        lat = []
        for o in range(0, E, B):
            t0 = time.perf_counter()
            if kind == "separate":
                s.fold_device(src[o:], dst[o:], n=B)
                s.take_delta_records(rec, cap, cnt)
            elif kind == "fused":
                s.fold_take(ps + 8 * o, pd + 8 * o, B, rec, cap, cnt)
                lat.append(time.perf_counter() - t0)
                continue
            elif kind in ("rawptr", "fold_sync"):
                check(L.gs_fold_device(x._h, ps + 8 * o, pd + 8 * o, None, B, 1))
                if kind == "rawptr":
                    check(L.gs_take_delta_records(x._h, pr, cap, pc))
            x.sync()
            lat.append(time.perf_counter() - t0)
        lat = np.array(lat[8:]) * 1e6
        return np.percentile(lat, 50), np.percentile(lat, 99)

    for kind in ("separate", "rawptr", "fold_sync", "fused", "sync_only", "separate", "fused"):
        p50, p99 = run(kind)
        print("%-10s p50 %6.2f us  p99 %6.2f us" % (kind, p50, p99), flush=True)
    s.close()
    s2.close()


if __name__ == "__main__":
    main()
