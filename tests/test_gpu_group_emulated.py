"""GPU: the native group (include/gs_group.h) at 2-4 ranks on the box's one GPU.
RCCL refuses two ranks on one device, so the group's communicator is replaced by
the library's in-process emulation (gs_group_set_comm_api + tests/cpp/gs_fake_comm.cpp: host barriers + device
copies ordered by events) and every rank is a thread of this process driving its
own summary. Everything else -- staging, 16-/24-byte rows, count and data
collectives, the exchange-layout fold of real remote rows on the side stream, the
partitioned label pass, the binomial tree combine -- is the code bench.py runs at N
GPUs. Every replica (or rank 0 of the tree) must equal the oracle."""
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


@pytest.mark.parametrize("world,batch", [(2, 1 << 12), (3, 1 << 11), (4, 1 << 12)])
def test_delta_exchange_emulated_ranks(gs, oracle_mod, fake_comm, world, batch):
    import torch
    scale, n, B = 14, 1 << 18, batch
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    uid = gs.group_unique_id()
    per = n // world

    def rank(r):
        with gs.Summary("cc", capacity_hint=1 << 10) as s:  # small hint: growth during the exchange
            g = gs.Group(s, uid, world, r, B)
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
    sent = sum(res[r][2]["records_sent"] for r in range(world))
    for r, (v, lab, st, _) in enumerate(res):
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "rank %d replica" % r
        assert st["exchanges"] == (per + B - 1) // B
        # live rows only: every rank receives at most max-count rows per peer per exchange
        assert st["rows_received"] <= (world - 1) * per
    assert sent <= n
    parts = sorted(p for r in range(world) for p in res[r][3])
    assert parts == sorted(zip(ov.tolist(), olab.tolist()))


_BENCH_SHAPE = {}


@pytest.mark.parametrize("world,log_batch", [(2, 20), (4, 20), (2, 22)])
def test_bench_exchange_shape_emulated_ranks(gs, oracle_mod, fake_comm, world, log_batch):
    """bench.py's N-GPU shape at reduced scale: RMAT-20 (2^24 edges), 2^20-edge
    per-rank micro-batches and 2^22, a capacity hint of twice
    the vertex scale. Every replica equals the oracle."""
    import torch
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


@pytest.mark.parametrize("lag", [1, 2, 3])
@pytest.mark.parametrize("kind", ["cc", "signed"])
def test_data_lag_emulated_ranks(gs, oracle_mod, fake_comm, knobs, lag, kind):
    """The data lag (GS_TESTING_GROUP_DATA_LAG): the data half of exchange b - L is issued
    after own fold b is queued (L = 1, 2; the default is 2) or, at L = 3, before it.
    Every schedule leaves every replica equal to the oracle (CC labels; signed colouring
    and verdict, with a mid-shard odd cycle in the signed case), with small batches so
    that many exchanges are in flight."""
    import torch
    knobs(group_data_lag=lag)
    world, B = 4, 1 << 11
    n = 1 << 17
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    if kind == "cc":
        gs.gen_rmat(src, dst, 0, n, 14, 0x5EED0026, True)
    else:
        gs.gen_bip(src, dst, 0, n, 13, 0x5EED0B1B, inject=((5 << 13) + 99,))
    torch.cuda.synchronize()
    uid = gs.group_unique_id()
    per = n // world

    def rank(r):
        with gs.Summary(kind, capacity_hint=1 << 10) as s:  # small hint: growth during the exchange
            g = gs.Group(s, uid, world, r, B)
            g.fold_batches(src[r * per:], dst[r * per:], per, B)
            g.finish()
            res = s.labels() if kind == "cc" else s.colouring()
            g.close()
        return res

    res = _run_ranks(world, rank)
    if kind == "cc":
        ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
        for r, (v, lab) in enumerate(res):
            assert np.array_equal(v, ov) and np.array_equal(lab, olab), "rank %d replica" % r
    else:
        t = oracle_mod.bip_truth(src.cpu().numpy(), dst.cpu().numpy())
        assert not t[0]
        for r, (ok, *_rest) in enumerate(res):
            assert ok == t[0], "rank %d verdict" % r


@pytest.mark.parametrize("inject", [(), (1 << 15,), (5 << 12,), (2 << 15) + 777])
def test_signed_exchange_emulated_ranks(gs, oracle_mod, fake_comm, inject):
    """inject (1 << 15) is the first edge of rank 1's shard (its endpoints are new
    there, so it travels as a hook record); (5 << 12) and (2 << 15) + 777 sit in the
    MIDDLE of a shard, where the injected same-side edge joins vertices that rank
    already connected: the odd cycle is found without any record, and only the count
    word's failure bit tells the other replicas."""
    import torch
    world, n, B = 3, 3 << 15, 1 << 12
    if not isinstance(inject, tuple):
        inject = (inject,)
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, n, 12, 0x5EED0B1B, inject=inject)
    torch.cuda.synchronize()
    uid = gs.group_unique_id()
    per = n // world

    def rank(r):
        with gs.Summary("signed", capacity_hint=1 << 12) as s:
            g = gs.Group(s, uid, world, r, B)
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
def test_tree_combine_emulated_ranks(gs, oracle_mod, fake_comm, kind, world):
    import torch
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


def test_eight_ranks_many_hw_queues_subprocess():
    """8 emulated ranks with 32 hardware queues (real concurrency between the own
    folds, the remote folds on the apply stream and the comm streams), 16 exchanges
    per rank per pass, 2 passes with a reset between: every replica equals the oracle
    after every pass. GPU_MAX_HW_QUEUES must be set before HIP starts, hence a child
    process. Regression: with highest-priority comm streams one XCD's share of some
    own-fold launches was lost here (gs_group.cpp create_comm_stream)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="32")
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "emu_check.py"), "--ranks", "8",
                        "--log-batch", "17", "--passes", "2"], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "all replicas equal the oracle" in r.stdout, r.stdout[-3000:] + r.stderr[-2000:]


def test_order_check_catches_a_misordered_rank(gs):
    """the emulation's order check itself. Two rank threads join a count
    and a data communicator and issue one collective on each; rank 1 in the other order makes
    every collective fail (each rank waits on the communicator the other is not in: a timeout,
    or an order-hash mismatch where they meet with different histories) instead of hanging --
    the condition that deadlocked an earlier build under RCCL. In order: all succeed."""
    import ctypes
    F = gs.fake_comm()
    errs = (ctypes.c_int * 4)()
    assert F.gs_fake_comm_selftest(0, 2000, errs) == 0
    assert list(errs) == [0, 0, 0, 0]
    assert F.gs_fake_comm_selftest(1, 500, errs) == 0
    assert all(e in (90, 91) for e in errs), list(errs)  # kErrOrder / kErrTimeout
