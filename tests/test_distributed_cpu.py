"""CPU (gloo, world_size 2 and 3): the multi-GPU combine protocol of
gelly-streaming_amd/distributed.py. Each rank folds its share of every global
micro-batch and exchanges its structural delta; afterwards every rank's replica
must equal the whole stream folded by the oracle (bit-exact canonical labels).

The device summary is replaced by `ModelReplica`, a CPU model of the C-ABI delta
contract (include/gs_summary.h: gs_set_delta_tracking / gs_delta_capacity /
gs_delta_stage / gs_fold_exchange_device): self-loop-only new vertices as
(v, v, 0), successful hooks as (root, new parent, parity); the stage writes every
record and a count word, the exchange fold reads block r's first counts[r] rows."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class ModelReplica:
    """Union-find with min-key hooking and delta recording (test model of the
    device replica: records are hooks (root, new parent, 0) and self-loop-only
    new vertices (v, v, 0))."""

    def __init__(self, capacity):
        self.parent = {}
        self.track = False
        self.delta = []
        self.capacity = capacity  # records one batch can produce (<= 1 per edge)

    def _find(self, v):
        while self.parent[v] != v:
            self.parent[v] = self.parent[self.parent[v]]
            v = self.parent[v]
        return v

    def _touch(self, v, self_loop):
        if v not in self.parent:
            self.parent[v] = v
            # only a new vertex seen through a self-loop gets its own record; any
            # other new vertex is named by a hook record
            if self.track and self_loop:
                self.delta.append((v, v, 0))

    def fold_device(self, src, dst, n=None, w=None, stride=1):
        s = src[:n].tolist()
        d = dst[:n].tolist()
        for a, b in zip(s, d):
            self._touch(a, a == b)
            self._touch(b, a == b)
            ra, rb = self._find(a), self._find(b)
            if ra == rb:
                continue
            hi, lo = (ra, rb) if ra > rb else (rb, ra)
            self.parent[hi] = lo
            if self.track:
                self.delta.append((hi, lo, 0))

    def set_delta_tracking(self, on=True):
        self.track = bool(on)
        self.delta = []

    def delta_capacity(self):
        return self.capacity

    def delta_stage(self, send, cap, count, width=3):
        """gs_delta_stage: every record into rows 0.., the count into `count`."""
        assert cap >= self.capacity and len(self.delta) <= cap
        if self.delta:
            send[:len(self.delta), :3] = torch.tensor(self.delta, dtype=torch.int64)
        count.fill_(len(self.delta))
        self.delta = []

    def fold_exchange(self, recv, counts, world, rows, skip_rank, width=3):
        saved = self.track
        self.track = False
        for r in range(world):
            if r == skip_rank:
                continue
            live = int(counts[r]) & ((1 << 62) - 1)
            rec = recv[r * rows:r * rows + live]
            rec = rec[(rec[:, 2] & 0x80) == 0]
            self.fold_device(rec[:, 0], rec[:, 1], n=len(rec))
        self.track = saved

    def sync(self):
        pass

    def labels(self):
        vs = sorted(self.parent)
        return np.array(vs, np.int64), np.array([self._find(v) for v in vs], np.int64)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, src, dst, batch, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import gsamd  # noqa: F401  (registers gelly_streaming_amd)
    from gelly_streaming_amd.distributed import DeltaExchangeFold

    rep = ModelReplica(batch)
    x = DeltaExchangeFold(rep, batch, torch.device("cpu"))
    s = torch.from_numpy(src)
    d = torch.from_numpy(dst)
    g = batch * world
    for o in range(0, len(src), g):  # global micro-batch: rank r folds slice r
        lo = o + rank * batch
        n = max(0, min(batch, len(src) - lo))
        x.step(s[lo:], d[lo:], n)
    x.finish()
    v, lab = rep.labels()
    out[rank] = (v.tolist(), lab.tolist(), x.rows_received, x.live_received)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 256), (3, 256), (2, 100), (3, 1000)])
def test_delta_exchange_gloo(oracle_mod, world, batch):
    src, dst = oracle_mod.rmat_edges(0x5EED0026, 12, 0, 1 << 13, True)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), src, dst, batch, out), nprocs=world, join=True)
    ov, olab = oracle_mod.cc_labels(src, dst)
    for r in range(world):
        v, lab, rows, live = out[r]
        assert v == ov.tolist(), "rank %d vertex set" % r
        assert lab == olab.tolist(), "rank %d labels" % r
        assert 0 < live <= rows  # only max-count rows per rank move: padding <= rows - live


# ---------------------------------------------------------------- owner-partitioned combine
class ModelForest:
    """Min-key union-find with parity -- the device forest's contract (every root is the
    minimum id of its tree; a hook records the root it moved) -- plus the partitioned
    combine's export state: insertion order, the mark of the previous export, the roots
    handed out as labels."""

    def __init__(self, signed):
        self.signed = signed
        self.parent, self.par = {}, {}
        self.bad = False
        self.order, self.mark = [], 0
        self.hooked, self.exported = [], set()

    def _touch(self, v):
        if v not in self.parent:
            self.parent[v] = v
            self.par[v] = 0
            self.order.append(v)

    def find(self, v):
        if v not in self.parent:
            return None
        path, p = [], 0
        while self.parent[v] != v:
            path.append(v)
            p ^= self.par[v]
            v = self.parent[v]
        root, acc = v, p
        for x in path:  # full compression with composed parities
            q = self.par[x]
            self.parent[x], self.par[x] = root, acc
            acc ^= q
        return root, p

    def fold(self, a, b, w=1):
        self._touch(a)
        self._touch(b)
        if a == b:
            return  # a self-loop adds its vertex and never fails (BipartitenessCheck.java:58-59)
        w = w if self.signed else 0
        (ra, pa), (rb, pb) = self.find(a), self.find(b)
        if ra == rb:
            if self.signed and (pa ^ pb) != w:
                self.bad = True
            return
        hi, lo = (ra, rb) if ra > rb else (rb, ra)
        self.parent[hi], self.par[hi] = lo, pa ^ pb ^ w
        self.hooked.append(hi)

    def export_new(self):
        rows = []
        for v in self.order[self.mark:]:
            root, p = self.find(v)
            self.exported.add(root)
            rows.append((v, root, p))
        self.mark = len(self.order)
        a = np.array(rows, np.int64).reshape(-1, 3)
        return a[:, 0], a[:, 1], a[:, 2]

    def hooked_exported(self):
        rows = []
        for a in self.hooked:
            if a in self.exported:
                root, p = self.find(a)
                self.exported.add(root)
                rows.append((a, root, p))
        self.hooked = []
        r = np.array(rows, np.int64).reshape(-1, 3)
        return r[:, 0], r[:, 1], r[:, 2]

    def failed(self):
        return self.bad

    def fail(self):
        self.bad = True


def _part_worker(rank, world, port, src, dst, window, signed, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import gsamd  # noqa: F401  (registers gelly_streaming_amd)
    from gelly_streaming_amd.distributed import PartitionedLabelCombine

    local, forest = ModelForest(signed), ModelForest(signed)
    x = PartitionedLabelCombine(local, forest)
    per = len(src) // world
    slices = []
    for w0 in range(0, per, window):
        for i in range(rank * per + w0, rank * per + min(per, w0 + window)):
            local.fold(int(src[i]), int(dst[i]))
        x.combine()
        v, lab, par = x.labels()
        slices.append((v.tolist(), lab.tolist(), par.tolist()))
    out[rank] = (slices, x.ok(), x.rows_owned)
    dist.barrier()
    dist.destroy_process_group()


def _merge_slices(out, world, k):
    from gelly_streaming_amd.distributed import part_owner
    v, lab, par = [], [], []
    for r in range(world):
        sv, sl, sp = out[r][0][k]
        assert all(int(o) == r for o in part_owner(np.array(sv, np.int64), world)), "rank %d owns its slice" % r
        v += sv
        lab += sl
        par += sp
    o = np.argsort(np.array(v, np.int64), kind="stable")
    return np.array(v, np.int64)[o], np.array(lab, np.int64)[o], np.array(par, np.int64)[o]


@pytest.mark.parametrize("world,window", [(2, 512), (3, 300), (5, 4096)])
def test_partitioned_combine_gloo_cc(oracle_mod, world, window):
    """DESIGN.md 5b over gloo: after EVERY combine the ranks' owned slices together equal the
    oracle's labels of the prefix folded so far (every rank's first windows)."""
    import gsamd  # noqa: F401
    src, dst = oracle_mod.rmat_edges(0x5EED0026, 11, 0, 3 * 5 * 1024, True)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_part_worker, args=(world, _free_port(), src, dst, window, False, out), nprocs=world, join=True)
    per = len(src) // world
    for k, w0 in enumerate(range(0, per, window)):
        idx = np.concatenate([np.arange(r * per, r * per + min(per, w0 + window)) for r in range(world)])
        ov, olab = oracle_mod.cc_labels(src[idx], dst[idx])
        v, lab, _ = _merge_slices(out, world, k)
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "combine %d" % k


@pytest.mark.parametrize("world,inject", [(2, ()), (4, ()), (3, (5000,))])
def test_partitioned_combine_gloo_signed(oracle_mod, world, inject):
    import gsamd  # noqa: F401
    src, dst = oracle_mod.bip_edges(0x5EED0B1B, 9, 0, 3 * 4 * 1024, inject)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_part_worker, args=(world, _free_port(), src, dst, 1024, True, out), nprocs=world, join=True)
    ok, comp, tv, sign = oracle_mod.bip_truth(src, dst)
    assert ok == (not inject)
    for r in range(world):
        assert out[r][1] == ok, "rank %d verdict" % r
    if ok:
        v, lab, par = _merge_slices(out, world, len(out[0][0]) - 1)
        o = np.argsort(tv, kind="stable")
        assert np.array_equal(v, tv[o]) and np.array_equal(lab, comp[o])
        assert np.array_equal(1 - par, sign[o].astype(np.int64))
