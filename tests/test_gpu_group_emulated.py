"""GPU: the native group (include/gs_group.h) at 2-4 ranks on the box's one GPU.
RCCL refuses two ranks on one device, so the group's communicator is replaced by
the library's in-process emulation (GS_GROUP_FAKE_COMM=1: host barriers + device
copies ordered by events) and every rank is a thread of this process driving its
own summary. Everything else -- staging, 16-/24-byte rows, the exchange-layout
fold of real remote rows on the side stream, header-driven retune, backlog drain,
partitioned label pass, the binomial tree combine -- is the code bench.py runs at
N GPUs. Every replica (or rank 0 of the tree) must equal the oracle."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run_ranks(world, body):
    out, errs = [None] * world, []

    def wrap(r):
        try:
            out[r] = body(r)
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs.append((r, e))

    ts = [threading.Thread(target=wrap, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    assert not errs, errs
    return out


@pytest.mark.parametrize("lanes", ["0", "1"])
@pytest.mark.parametrize("world,first_cap,retune", [(2, 0, "4"), (3, 256, "2"), (4, 64, "1")])
def test_delta_exchange_emulated_ranks(gs, oracle_mod, monkeypatch, world, first_cap, retune, lanes):
    """lanes=1: each rank's own tracked folds alternate over two lane streams and two
    delta sets (GS_GROUP_LANES), the stage of exchange b on fold b's lane."""
    import torch
    monkeypatch.setenv("GS_GROUP_FAKE_COMM", "1")
    monkeypatch.setenv("GS_GROUP_LANES", lanes)
    monkeypatch.setenv("GS_GROUP_RETUNE", retune)
    scale, n, B = 14, 1 << 18, 1 << 12
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    uid = gs.group_unique_id()
    per = n // world

    def rank(r):
        with gs.Summary("cc", capacity_hint=1 << 10) as s:  # small hint: growth during the exchange
            g = gs.Group(s, uid, world, r, B, first_cap)
            g.fold_batches(src[r * per:], dst[r * per:], per, B)
            g.finish()
            st = g.stats()
            v, lab = s.labels()
            # partitioned label pass: this rank's slot range
            m = s.num_vertices() + 1
            pv = torch.empty(m, dtype=torch.int64, device="cuda")
            pl = torch.empty(m, dtype=torch.int64, device="cuda")
            k = s.export_labels_part_device(r, world, pv, pl)
            part = sorted(zip(pv[:k].tolist(), pl[:k].tolist()))
            g.close()
        return v, lab, st, part

    res = _run_ranks(world, rank)
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    for r, (v, lab, st, _) in enumerate(res):
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "rank %d replica" % r
        assert st["exchanges"] >= per // B
    parts = sorted(p for r in range(world) for p in res[r][3])
    assert parts == sorted(zip(ov.tolist(), olab.tolist()))


_BENCH_SHAPE = {}


@pytest.mark.parametrize("world,log_batch", [(2, 22), (4, 21)])
def test_bench_exchange_shape_emulated_ranks(gs, oracle_mod, monkeypatch, world, log_batch):
    """bench.py's N-GPU defaults at reduced scale: RMAT-20 (2^24 edges), 2^21-2^22-edge
    exchanges per rank, a capacity hint of twice the vertex scale, the default first
    capacity and knobs. Every replica equals the oracle."""
    import torch
    monkeypatch.setenv("GS_GROUP_FAKE_COMM", "1")
    scale, n, B = 20, 1 << 24, 1 << log_batch
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    if "oracle" not in _BENCH_SHAPE:
        _BENCH_SHAPE["oracle"] = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    ov, olab = _BENCH_SHAPE["oracle"]
    uid = gs.group_unique_id()
    per = n // world

    def rank(r):
        with gs.Summary("cc", capacity_hint=1 << (scale + 1)) as s:
            g = gs.Group(s, uid, world, r, B)
            g.fold_batches(src[r * per:], dst[r * per:], per, B)
            g.finish()
            st = g.stats()
            v, lab = s.labels()
            g.close()
        return v, lab, st

    for r, (v, lab, st) in enumerate(_run_ranks(world, rank)):
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "rank %d replica" % r
        assert st["exchanges"] >= per // B


@pytest.mark.parametrize("lanes", ["0", "1"])
@pytest.mark.parametrize("inject", [(), (1 << 15,)])
def test_signed_exchange_emulated_ranks(gs, oracle_mod, monkeypatch, inject, lanes):
    import torch
    monkeypatch.setenv("GS_GROUP_FAKE_COMM", "1")
    monkeypatch.setenv("GS_GROUP_LANES", lanes)
    monkeypatch.setenv("GS_GROUP_RETUNE", "2")
    world, n, B = 3, 3 << 15, 1 << 12
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, n, 12, 0x5EED0B1B, inject=inject)
    torch.cuda.synchronize()
    uid = gs.group_unique_id()
    per = n // world

    def rank(r):
        with gs.Summary("signed", capacity_hint=1 << 12) as s:
            g = gs.Group(s, uid, world, r, B, 512)
            g.fold_batches(src[r * per:], dst[r * per:], per, B)
            g.finish()
            res = s.colouring()
            g.close()
        return res

    res = _run_ranks(world, rank)
    t = oracle_mod.bip_truth(src.cpu().numpy(), dst.cpu().numpy())
    assert t[0] == (not inject)
    for r, (ok, comp, v, sign) in enumerate(res):
        assert ok == t[0], "rank %d verdict" % r
        if ok:
            assert np.array_equal(comp, t[1]) and np.array_equal(v, t[2]) and np.array_equal(sign, t[3])


@pytest.mark.parametrize("kind,world", [("cc", 3), ("cc", 4), ("signed", 3)])
def test_tree_combine_emulated_ranks(gs, oracle_mod, monkeypatch, kind, world):
    import torch
    monkeypatch.setenv("GS_GROUP_FAKE_COMM", "1")
    n = 1 << 16
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    if kind == "cc":
        gs.gen_rmat(src, dst, 0, n, 13, 0x5EED0026, True)
    else:
        gs.gen_bip(src, dst, 0, n, 11, 0x5EED0B1B)
    torch.cuda.synchronize()
    uid = gs.group_unique_id()
    bounds = [r * n // world for r in range(world + 1)]

    def rank(r):
        with gs.Summary(kind, capacity_hint=1 << 10) as s:
            g = gs.Group(s, uid, world, r, 0)  # tree-only group
            lo, hi = bounds[r], bounds[r + 1]
            s.fold_device(src[lo:], dst[lo:], n=hi - lo)
            g.tree_combine()
            res = s.labels() if kind == "cc" else s.colouring()
            g.close()
        return res

    res = _run_ranks(world, rank)
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    if kind == "cc":
        ov, olab = oracle_mod.cc_labels(hs, hd)
        assert np.array_equal(res[0][0], ov) and np.array_equal(res[0][1], olab)
    else:
        ok, comp, v, sign = res[0]
        t = oracle_mod.bip_truth(hs, hd)
        assert ok == t[0] and ok
        assert np.array_equal(comp, t[1]) and np.array_equal(v, t[2]) and np.array_equal(sign, t[3])
