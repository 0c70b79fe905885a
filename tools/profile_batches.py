"""Per-micro-batch kernel times of the streaming CC fold (HIP events on the
summary's stream). Usage: python tools/profile_batches.py [--scale 26] [--log-batch 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--scale", type=int, default=26)
p.add_argument("--log-batch", type=int, default=20)
p.add_argument("--seed", type=lambda x: int(x, 0), default=0x5EED0026)
p.add_argument("--out", default="gpurun_out/batches.json")
a = p.parse_args()
E = 16 << a.scale
B = 1 << a.log_batch
s = gs.Summary("cc", capacity_hint=1 << a.scale)
src = torch.empty(E, dtype=torch.int64, device="cuda")
dst = torch.empty(E, dtype=torch.int64, device="cuda")
gs.gen_rmat(src, dst, 0, E, a.scale, a.seed, True, stream=s.stream)
s.sync()
rows = []
tot = {"fold": 0.0, "hook": 0.0}
for b in range(E // B):
    s.set_profiling(True)
    s.fold_device(src[b * B:], dst[b * B:], n=B)
    s.sync()
    f = s.kernel_stats("fold")[1]
    h = s.kernel_stats("hook")[1]
    tot["fold"] += f
    tot["hook"] += h
    if b < 8 or (b & (b - 1)) == 0 or b == E // B - 1:
        rows.append({"batch": b, "fold_us": round(f * 1e3, 1), "hook_us": round(h * 1e3, 1), "nv": s.num_vertices()})
        print(rows[-1], flush=True)
s.set_profiling(False)
print(json.dumps({"total_fold_ms": tot["fold"], "total_hook_ms": tot["hook"], "batches": E // B}))
os.makedirs(os.path.dirname(a.out), exist_ok=True)
with open(a.out, "w") as f:
    json.dump({"rows": rows, "total": tot}, f)
