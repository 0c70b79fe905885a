"""Per-batch hook statistics with the debug-counter build:
  make -C gelly-streaming_amd debug
  GS_LIB=gelly-streaming_amd/lib_debug/libgs_summary.so python tools/hook_stats.py
prints, for the first BATCHES 2^20-edge batches of RMAT-26: fold time (HIP events),
hook calls, hook-loop iterations and failed CASes (deltas per batch)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

if os.environ.get("GS_LIB"):
    gs.LIB_PATH = os.path.join(ROOT, os.environ["GS_LIB"])
B = 1 << 20
nb = int(os.environ.get("BATCHES", "8"))
s = gs.Summary("cc", capacity_hint=1 << 25)
src = torch.empty(nb * B, dtype=torch.int64, device="cuda")
dst = torch.empty(nb * B, dtype=torch.int64, device="cuda")
gs.gen_rmat(src, dst, 0, nb * B, 26, 0x5EED0026, True, stream=s.stream)
s.sync()
prev = s.counters()
print("batch fold_us vertices hooks hook_iters cas_fail")
for b in range(nb):
    s.set_profiling(True)
    s.fold_device(src[b * B:], dst[b * B:], n=B)
    s.sync()
    f = s.kernel_stats("fold")[1] * 1e3
    c = s.counters()
    print(b, round(f, 1), c["vertices"], c["hooks"] - prev["hooks"], c["hook_iters"] - prev["hook_iters"],
          c["cas_fail"] - prev["cas_fail"], flush=True)
    prev = c
