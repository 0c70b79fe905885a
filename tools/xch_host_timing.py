"""Host-time breakdown of DeltaExchangeFold.step at one rank (nccl, world 1) on RMAT-26.
python tools/xch_host_timing.py [--log-batch 20] [--batches 512]"""
import argparse
import os
import sys
import time
from collections import defaultdict

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402
from gelly_streaming_amd.distributed import DeltaExchangeFold  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--log-batch", type=int, default=20)
p.add_argument("--batches", type=int, default=512)
a = p.parse_args()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29544")
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
B = 1 << a.log_batch
E = B * a.batches
s = gs.Summary("cc", capacity_hint=1 << 25)
src = torch.empty(E, dtype=torch.int64, device=dev)
dst = torch.empty(E, dtype=torch.int64, device=dev)
gs.gen_rmat(src, dst, 0, E, 26, 0x5EED0026, True, stream=s.stream)
s.sync()
x = DeltaExchangeFold(s, B, dev)
acc = defaultdict(float)


def timed(name, fn):
    def w(*args, **kw):
        t = time.perf_counter()
        r = fn(*args, **kw)
        acc[name] += time.perf_counter() - t
        return r
    return w


x._after = timed("after", x._after)
x._exchange = timed("exchange", x._exchange)
x._apply = timed("apply", x._apply)
s.fold_device = timed("fold_device", s.fold_device)
s.delta_stage = timed("delta_stage", s.delta_stage)
s.fold_exchange = timed("fold_exchange", s.fold_exchange)
for rep in range(2):
    acc.clear()
    s.reset()
    s.set_delta_tracking(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in range(a.batches):
        x.step(src[b * B:], dst[b * B:], B)
    th = time.perf_counter() - t0
    x.finish()
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
print("host loop %.1f ms, wall %.1f ms, per batch host %.1f us" % (th * 1e3, tw * 1e3, th * 1e6 / a.batches))
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    print("  %-12s %8.1f us/batch" % (k, v * 1e6 / a.batches))
dist.destroy_process_group()
