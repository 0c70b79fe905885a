"""Host vs device time of the native group exchange loop at one rank (RMAT-26):
is gs_group_fold_batches_device host-bound? python tools/xch_native_timing.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402

B = int(os.environ.get("BATCH", str(1 << 20)))
nb = int(os.environ.get("BATCHES", "256"))
s = gs.Summary("cc", capacity_hint=1 << 25)
src = torch.empty(nb * B, dtype=torch.int64, device="cuda")
dst = torch.empty(nb * B, dtype=torch.int64, device="cuda")
gs.gen_rmat(src, dst, 0, nb * B, 26, 0x5EED0026, True, stream=s.stream)
s.sync()
g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
for rep in range(2):
    s.reset()
    t0 = time.perf_counter()
    g.fold_batches(src, dst, nb * B, B)
    t1 = time.perf_counter()
    g.finish()
    t2 = time.perf_counter()
    print("rep %d: host enqueue %.1f us/batch, total %.1f us/batch" % (rep, (t1 - t0) * 1e6 / nb, (t2 - t0) * 1e6 / nb),
          flush=True)
g.close()
