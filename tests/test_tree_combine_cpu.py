"""CPU (gloo, world_size 2/3/4/5): the log-depth tree combine of per-rank partial
summaries (gelly_streaming_amd.distributed.tree_combine; the reference's
SummaryTreeReduce, SummaryTreeReduce.java:68-123). Each rank folds a contiguous
shard of the stream into its own partial; after the tree, rank 0 must hold the
whole stream: CC labels bit-exact vs the oracle's DisjointSet, and for the signed
kind the verdict and colouring equal the truth (sticky AND over partials).

The device summary is replaced by `ModelPartial`, a CPU model of the export /
combine-exported contract (include/gs_summary.h: gs_export_labels_device emits
(v, min-key label, parity relative to the label); gs_combine_exported_device folds
union(v, label) with that parity and ANDs the verdict)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class ModelPartial:
    device = torch.device("cpu")

    def __init__(self, signed):
        self.signed = signed
        self.parent = {}  # v -> (parent, parity to parent)
        self.failed = False

    def _find(self, v):
        p = 0
        while self.parent[v][0] != v:
            u, q = self.parent[v]
            p ^= q
            v = u
        return v, p

    def fold(self, src, dst, w=None):
        for i, (a, b) in enumerate(zip(src, dst)):
            for x in (a, b):
                self.parent.setdefault(x, (x, 0))
            need = 1 if w is None else int(w[i])
            if a == b:
                continue  # a self-loop adds the vertex and never fails (BipartitenessCheck.java:58-59)
            ra, pa = self._find(a)
            rb, pb = self._find(b)
            if ra == rb:
                if self.signed and pa ^ pb != need:
                    self.failed = True
                continue
            hi, lo = (ra, rb) if ra > rb else (rb, ra)
            self.parent[hi] = (lo, pa ^ pb ^ need)

    def num_vertices(self):
        return len(self.parent)

    def ok(self):
        return not self.failed

    def export_labels_device(self, v, lab, par):
        vs = sorted(self.parent)
        for i, x in enumerate(vs):
            r, p = self._find(x)
            v[i], lab[i], par[i] = x, r, p
        return len(vs)

    def combine_exported_device(self, v, lab, par, n, failed):
        if failed:
            self.failed = True
            return
        self.fold(v[:n].tolist(), lab[:n].tolist(), par[:n].tolist())

    def sync(self):
        pass


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, src, dst, signed, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import gsamd  # noqa: F401  (registers gelly_streaming_amd)
    from gelly_streaming_amd.distributed import tree_combine

    m = ModelPartial(signed)
    lo, hi = rank * len(src) // world, (rank + 1) * len(src) // world
    m.fold(src[lo:hi].tolist(), dst[lo:hi].tolist())
    holds = tree_combine(m, None)
    if rank == 0:
        n = m.num_vertices()
        v = torch.empty(n, dtype=torch.int64)
        lab = torch.empty(n, dtype=torch.int64)
        par = torch.empty(n, dtype=torch.uint8)
        m.export_labels_device(v, lab, par)
        out[rank] = (holds, m.ok(), v.tolist(), lab.tolist(), par.tolist())
    else:
        out[rank] = (holds,)
    dist.barrier()
    dist.destroy_process_group()


def _run(src, dst, world, signed):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), src, dst, signed, out), nprocs=world, join=True)
    assert out[0][0] and not any(out[r][0] for r in range(1, world))
    return out[0][1:]


@pytest.mark.parametrize("world", [2, 3, 4, 5])
def test_tree_combine_cc_gloo(oracle_mod, world):
    src, dst = oracle_mod.rmat_edges(0x5EED0026, 11, 0, 1 << 12, True)
    ok, v, lab, _ = _run(src, dst, world, False)
    ov, olab = oracle_mod.cc_labels(src, dst)
    assert v == ov.tolist() and lab == olab.tolist()


@pytest.mark.parametrize("inject", [(), (1500,)])
def test_tree_combine_bipartite_gloo(oracle_mod, inject):
    src, dst = oracle_mod.bip_edges(0x5EED0B1B, 9, 0, 1 << 12, inject)
    ok, v, lab, par = _run(src, dst, 3, True)
    tok, tcomp, tv, tsign = oracle_mod.bip_truth(src, dst)
    assert ok == tok
    if ok:  # sign(v) = (parity(v) == parity(min)); the label IS the min, parity relative to it
        got = sorted(zip(lab, v, [1 - p for p in par]))
        assert got == sorted(zip(tcomp.tolist(), tv.tolist(), tsign.tolist()))
