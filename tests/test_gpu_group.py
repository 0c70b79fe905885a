"""GPU: the native RCCL group (include/gs_group.h) at one rank: fold + stage +
count all-gather + live-row data all-gather + side-stream apply.
(Several ranks need several GPUs: RCCL refuses two ranks on one device; the
multi-rank protocol itself is covered by test_gpu_distributed.py / the gloo tests.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("self_apply,batch", [(0, 1 << 13), (1, 1 << 13), (1, 1 << 12)])
def test_group_single_rank_matches_oracle(gs, oracle_mod, knobs, self_apply, batch):
    """self_apply: the rank also folds its own gathered rows (16-B CC rows, exchange
    layout from the gathered count words, applied one exchange late on the side
    stream) -- the remote-fold path, exercised at one rank; folding a delta twice is
    idempotent, so any mis-parsed row would show in the labels."""
    import torch
    knobs(group_self_apply=self_apply)
    n, B = 1 << 17, batch
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, 15, 0x5EED0026, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 15) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
        for i in range(0, n, B):
            g.fold_device(src[i:], dst[i:], B)
        with pytest.raises(gs.GSError):  # n above batch_edges is refused up front
            g.fold_device(src, dst, B + 1)
        g.finish()
        st = g.stats()
        assert st["exchanges"] == n // B
        assert 0 < st["records_sent"] <= n
        v, lab = s.labels()
        g.close()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_group_fold_batches_native_loop(gs, oracle_mod, knobs):
    """gs_group_fold_batches_device == the per-batch calls (ragged last batch)."""
    import torch
    knobs(group_self_apply=1)
    n, B = (1 << 16) + 777, 1 << 12
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, 14, 0x5EED0026, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 14) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
        g.fold_batches(src, dst, n, B)
        g.finish()
        assert g.stats()["exchanges"] >= (n + B - 1) // B
        v, lab = s.labels()
        g.close()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


@pytest.mark.parametrize("inject", [(), (1 << 15,)])
def test_group_signed_rows_self_apply(gs, oracle_mod, knobs, inject):
    """Signed summary in a group: 24-B rows {a, b, parity}; the rank folds its own
    gathered rows back (GS_TESTING_GROUP_SELF_APPLY) -- verdict and colouring must equal
    the truth."""
    import torch
    knobs(group_self_apply=1)
    n, B = 1 << 16, 1 << 12
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, n, 12, 0x5EED0B1B, inject=inject)
    torch.cuda.synchronize()
    with gs.Summary("signed", capacity_hint=1 << 13) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
        for i in range(0, n, B):
            g.fold_device(src[i:], dst[i:], B)
        g.finish()
        ok, comp, v, sign = s.colouring()
        g.close()
    t = oracle_mod.bip_truth(src.cpu().numpy(), dst.cpu().numpy())
    assert ok == t[0] and ok == (not inject)
    if ok:
        assert np.array_equal(comp, t[1]) and np.array_equal(v, t[2]) and np.array_equal(sign, t[3])


@pytest.mark.parametrize("kind", ["cc", "signed"])
def test_combine_exported_device_equals_combine(gs, oracle_mod, kind):
    """gs_combine_exported_device (the receiving half of the tree combine) folds
    another summary's exported arrays: same result as gs_combine."""
    import torch
    n = 1 << 15
    if kind == "cc":
        s, d = oracle_mod.rmat_edges(0x5EED0026, 12, 0, n, True)
    else:
        s, d = oracle_mod.bip_edges(0x5EED0B1B, 11, 0, n)
    h = n // 2
    with gs.Summary(kind, capacity_hint=64) as a, gs.Summary(kind, capacity_hint=64) as b, \
            gs.Summary(kind, capacity_hint=64) as c:
        a.fold(s[:h], d[:h])
        b.fold(s[h:], d[h:])
        c.fold(s[h:], d[h:])
        m = a.num_vertices() + 1
        v = torch.empty(m, dtype=torch.int64, device="cuda")
        lab = torch.empty(m, dtype=torch.int64, device="cuda")
        par = torch.empty(m, dtype=torch.uint8, device="cuda")
        got = a.export_labels_device(v, lab, par)
        b.combine_exported_device(v, lab, par, got, failed=not a.ok())
        c.combine(a)
        if kind == "cc":
            ov, olab = oracle_mod.cc_labels(s, d)
            for x in (b, c):
                xv, xl = x.labels()
                assert np.array_equal(xv, ov) and np.array_equal(xl, olab)
        else:
            t = oracle_mod.bip_truth(s, d)
            for x in (b, c):
                ok, comp, xv, sign = x.colouring()
                assert ok == t[0] and ok
                assert np.array_equal(comp, t[1]) and np.array_equal(xv, t[2]) and np.array_equal(sign, t[3])
        b.combine_exported_device(v, lab, par, 0, failed=True)
        assert kind == "cc" or not b.ok()


def test_tree_only_group_single_rank(gs, oracle_mod):
    """batch_edges 0: a tree-combine-only group (no exchange buffers, tracking off);
    at one rank the tree is empty and the summary is unchanged."""
    s, d = oracle_mod.rmat_edges(0x5EED0026, 12, 0, 1 << 14, True)
    with gs.Summary("cc", capacity_hint=1 << 12) as x:
        g = gs.Group(x, gs.group_unique_id(), 1, 0, 0)
        x.fold(s, d)  # tracking is off: no delta capacity limit applies
        g.tree_combine()
        with pytest.raises(gs.GSError):
            g.fold_device(None, None, 0)
        v, lab = x.labels()
        g.close()
    ov, olab = oracle_mod.cc_labels(s, d)
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_group_ramp_exchange_cadence(gs, oracle_mod, knobs):
    """gs_group_set_ramp: the first `ramp` edges after create / finish are exchanged
    every `ramp_batch` edges, the rest every `batch` (a self-applying rank folds its
    own rows back, so every exchange's rows are parsed); the ramp restarts after
    finish, bad arguments are refused."""
    import torch
    knobs(group_self_apply=1)
    n, B = 1 << 17, 1 << 14
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, 15, 0x5EED0026, True)
    torch.cuda.synchronize()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    with gs.Summary("cc", capacity_hint=1 << 15) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B)
        with pytest.raises(gs.GSError):
            g.set_ramp(1 << 15, B * 2)  # ramp batch above batch_edges
        g.set_ramp(1 << 15, 1 << 12)
        for p in range(2):  # the ramp restarts after finish
            s.reset()
            g.fold_batches(src, dst, n, B)
            g.finish()
            st = g.stats()
            # 2^15 edges in 2^12 exchanges (8), then 2^17 - 2^15 in 2^14 exchanges (6)
            assert st["exchanges"] == (p + 1) * (8 + 6)
            v, lab = s.labels()
            assert np.array_equal(v, ov) and np.array_equal(lab, olab)
        g.set_ramp(0)  # off: 2^17 / 2^14 exchanges
        s.reset()
        g.fold_batches(src, dst, n, B)
        g.finish()
        assert g.stats()["exchanges"] == 2 * 14 + 8
        g.close()
