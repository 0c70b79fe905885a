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
    x = DeltaExchangeFold(summ, batch, dev)
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


def _tree_worker(rank, world, port, kind, nedges, out):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import gsamd as gs
    from gelly_streaming_amd.distributed import tree_combine
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    src = torch.empty(nedges, dtype=torch.int64, device=dev)
    dst = torch.empty(nedges, dtype=torch.int64, device=dev)
    if kind == "cc":
        gs.gen_rmat(src, dst, 0, nedges, 13, 0x5EED0026, True)
    else:
        gs.gen_bip(src, dst, 0, nedges, 12, 0x5EED0B1B, inject=(nedges // 2,) if kind == "bip-odd" else ())
    torch.cuda.synchronize()
    summ = gs.Summary("cc" if kind == "cc" else "signed", device=0, capacity_hint=1 << 10)
    lo, hi = rank * nedges // world, (rank + 1) * nedges // world
    summ.fold_device(src[lo:], dst[lo:], n=hi - lo)
    holds = tree_combine(summ, None)
    if rank == 0:
        if kind == "cc":
            v, lab = summ.labels()
            out[rank] = (holds, v.tobytes(), lab.tobytes())
        else:
            ok, comp, v, sign = summ.colouring()
            out[rank] = (holds, ok, comp.tobytes(), v.tobytes(), sign.tobytes())
    else:
        out[rank] = (holds,)
    summ.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("cc", 2), ("cc", 3), ("bip", 3), ("bip-odd", 2)])
def test_tree_combine_ranks_share_one_gpu(oracle_mod, kind, world):
    """gelly_streaming_amd.distributed.tree_combine (SummaryTreeReduce) with real HIP
    partial summaries: rank 0 must end with the whole stream."""
    nedges = 1 << 16
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_tree_worker, args=(world, _free_port(), kind, nedges, out), nprocs=world, join=True)
    assert out[0][0] and not any(out[r][0] for r in range(1, world))
    if kind == "cc":
        s, d = oracle_mod.rmat_edges(0x5EED0026, 13, 0, nedges, True)
        ov, olab = oracle_mod.cc_labels(s, d)
        assert np.array_equal(np.frombuffer(out[0][1], np.int64), ov)
        assert np.array_equal(np.frombuffer(out[0][2], np.int64), olab)
    else:
        s, d = oracle_mod.bip_edges(0x5EED0B1B, 12, 0, nedges, (nedges // 2,) if kind == "bip-odd" else ())
        tok, tcomp, tv, tsign = oracle_mod.bip_truth(s, d)
        _, ok, comp, v, sign = out[0]
        assert ok == tok and ok == (kind == "bip")
        if ok:
            assert np.array_equal(np.frombuffer(comp, np.int64), tcomp)
            assert np.array_equal(np.frombuffer(v, np.int64), tv)
            assert np.array_equal(np.frombuffer(sign, np.uint8), tsign)
