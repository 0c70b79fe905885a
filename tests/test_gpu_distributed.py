"""GPU, 2 ranks on the box's one GPU (gloo transport, payload staged through host
memory): every rank folds its half of each global micro-batch into its own HIP
summary and applies the other rank's delta (gelly_streaming_amd.distributed).
Both replicas must equal the oracle on the whole stream. The nccl/RCCL transport
of the same code is exercised by bench.py --gpus N on a multi-GPU node."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, scale, nedges, batch, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import gsamd as gs
    from gelly_streaming_amd.distributed import DeltaExchangeFold
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    summ = gs.Summary("cc", device=0, capacity_hint=1 << scale)
    src = torch.empty(nedges, dtype=torch.int64, device=dev)
    dst = torch.empty(nedges, dtype=torch.int64, device=dev)
    gs.gen_rmat(src, dst, 0, nedges, scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    x = DeltaExchangeFold(summ, batch, dev, first_cap=batch // 64, retune=4)
    g = batch * world
    for o in range(0, nedges, g):
        lo = o + rank * batch
        n = max(0, min(batch, nedges - lo))
        x.step(src[lo:], dst[lo:], n)
    x.finish()
    v, lab = summ.labels()
    out[rank] = (v.tobytes(), lab.tobytes(), x.rows_received)
    summ.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_share_one_gpu(oracle_mod):
    scale, nedges, batch = 14, 1 << 18, 1 << 14
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), scale, nedges, batch, out), nprocs=2, join=True)
    s, d = oracle_mod.rmat_edges(0x5EED0026, scale, 0, nedges, True)
    ov, olab = oracle_mod.cc_labels(s, d)
    for r in range(2):
        vb, lb, exchanged = out[r]
        v = np.frombuffer(vb, np.int64)
        lab = np.frombuffer(lb, np.int64)
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "rank %d" % r
        assert exchanged > 0
