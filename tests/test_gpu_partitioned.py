"""GPU: the owner-partitioned group (include/gs_group.h gs_group_create_partitioned,
DESIGN.md section 5b) at 1-8 ranks on the box's one GPU, every rank a thread of this
process with its own local summary, collectives through the in-process emulation
(gs_group_set_comm_api + tests/cpp/gs_fake_comm.cpp, which also fails a collective whose
ranks issued the communicators' collectives in different orders). The union of the ranks'
owned slices must equal the oracle (CC labels = min id; signed: verdict, and colourings
against the truth) after EVERY combine -- windowed mode checks the prefix folded so far --
with small hints, so local tables rebuild mid-stream (the full re-export path)."""
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
        t.join(timeout=200)
    assert not any(t.is_alive() for t in ts), "a rank hung"
    assert not errs, errs
    return out


def _owner(v, n):
    """part_owner (csrc/gs_part.hpp) in numpy."""
    z = (np.asarray(v, np.int64).view(np.uint64) ^ np.uint64(0x5851F42D4C957F2D))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return ((z >> np.uint64(32)) % np.uint64(n)).astype(np.int64)


def _merge(slices, world):
    v = np.concatenate([s[0] for s in slices])
    lab = np.concatenate([s[1] for s in slices])
    for r, s in enumerate(slices):  # every rank emits only the vertices it owns
        assert np.all(_owner(s[0], world) == r), "rank %d emitted a vertex it does not own" % r
    o = np.argsort(v, kind="stable")
    extra = [np.concatenate([s[2] for s in slices])[o]] if len(slices[0]) > 2 else []
    return (v[o], lab[o], *extra)


@pytest.mark.parametrize("world,window,hint,pipe", [(1, 0, 1 << 14, 1), (2, 0, 1 << 8, 3), (3, 1 << 12, 1 << 8, 1),
                                                    (4, 1 << 11, 1 << 14, 3), (8, 1 << 12, 1 << 8, 3),
                                                    (8, 0, 1 << 14, 1)])
def test_partitioned_cc_every_combine_equals_oracle(gs, oracle_mod, fake_comm, world, window, hint, pipe):
    """(pipe 3: pipelined own folds -- tracked ones too in windowed mode -- joined by the combine)"""
    import torch
    scale, n = 14, 1 << 17
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    uid = gs.group_unique_id()
    per = n // world
    W = window or per
    nwin = (per + W - 1) // W
    barrier = threading.Barrier(world)
    got = {}

    def rank(r):
        with gs.Summary("cc", capacity_hint=hint) as s:  # small hints: the local table rebuilds mid-stream
            s.set_pipelining(pipe)
            g = gs.PartGroup(s, uid, world, r, 1 << scale, window)
            for w in range(nwin):
                lo, m = r * per + w * W, min(W, per - w * W)
                q = max(m // 4, 1)
                for o in range(0, m, q):  # four folds per window (they overlap on the lanes with pipe 3)
                    g.fold_device(src[lo + o:], dst[lo + o:], min(q, m - o))
                g.combine()
                got[(w, r)] = g.labels(1 << (scale + 1))
                barrier.wait()
            st = g.stats()
            g.close()
        return st

    stats = _run_ranks(world, rank)
    for w in range(nwin):  # the prefix: every rank's first w + 1 windows
        idx = np.concatenate([np.arange(r * per, r * per + min((w + 1) * W, per)) for r in range(world)])
        ov, olab = oracle_mod.cc_labels(hs[idx], hd[idx])
        v, lab = _merge([got[(w, r)] for r in range(world)], world)
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "combine %d" % w
    assert all(st["combines"] == nwin for st in stats)
    # the label forest holds a small fraction of the vertices
    assert stats[0]["label_forest_vertices"] <= len(ov)


@pytest.mark.parametrize("world,window,inject", [(2, 0, ()), (4, 1 << 12, ()), (3, 1 << 12, ((3 << 14) + 77,)),
                                                 (4, 0, ((1 << 15) + 5,)), (8, 1 << 11, ())])
def test_partitioned_signed_verdict_and_colouring(gs, oracle_mod, fake_comm, world, window, inject):
    import torch
    logside, n = 12, 3 << 15
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, n, logside, 0x5EED0B1B, inject=inject)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    uid = gs.group_unique_id()
    per = n // world
    W = window or per
    nwin = (per + W - 1) // W

    def rank(r):
        with gs.Summary("signed", capacity_hint=1 << 8) as s:
            g = gs.PartGroup(s, uid, world, r, 1 << (logside + 1), window)
            for w in range(nwin):
                lo = r * per + w * W
                g.fold_device(src[lo:], dst[lo:], min(W, per - w * W))
                g.combine()
            res = (g.ok(), g.labels(1 << (logside + 2), with_parity=True))
            g.close()
        return res

    res = _run_ranks(world, rank)
    ok, comp, tv, sign = oracle_mod.bip_truth(hs[:per * world], hd[:per * world])
    assert ok == (not inject)
    for r in range(world):
        assert res[r][0] == ok, "rank %d verdict" % r
    if ok:
        v, lab, par = _merge([res[r][1] for r in range(world)], world)
        o = np.argsort(tv, kind="stable")
        assert np.array_equal(v, tv[o]) and np.array_equal(lab, comp[o])
        assert np.array_equal(1 - par.astype(np.int64), sign[o].astype(np.int64))


def test_partitioned_extreme_ids_self_loops_and_idle_ranks(gs, oracle_mod, fake_comm):
    """INT64_MIN / INT64_MAX and negative ids, self-loops (a vertex with no other edge), and a
    rank that folds nothing in some windows; then a reset and a second pass."""
    import torch
    mn, mx = np.iinfo(np.int64).min, np.iinfo(np.int64).max
    a = np.array([mn, 5, -7, mx, 9, 9, 1 << 40, -(1 << 50), 3, mn + 1, 11, 12], np.int64)
    b = np.array([5, -7, 9, 1 << 40, 9, 3, -(1 << 50), mx, 3, mn, 12, 11], np.int64)
    world = 3
    uid = gs.group_unique_id()
    shards = [(a[:5], b[:5]), (a[5:5], b[5:5]), (a[5:], b[5:])]  # rank 1 folds nothing

    def rank(r):
        out = []
        with gs.Summary("cc", capacity_hint=4) as s:
            g = gs.PartGroup(s, uid, world, r, 64, 16)
            for _ in range(2):
                sa = torch.tensor(shards[r][0], dtype=torch.int64, device="cuda")
                sb = torch.tensor(shards[r][1], dtype=torch.int64, device="cuda")
                g.fold_device(sa, sb, len(shards[r][0]))
                g.combine()
                g.combine()  # an empty window
                out.append(g.labels(64))
                g.reset()
            g.close()
        return out

    res = _run_ranks(world, rank)
    ov, olab = oracle_mod.cc_labels(a, b)
    for p in range(2):
        v, lab = _merge([res[r][p] for r in range(world)], world)
        assert np.array_equal(v, ov) and np.array_equal(lab, olab), "pass %d" % p
