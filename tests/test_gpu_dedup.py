"""GPU: micro-batch dedup by hashing (gs_set_batch_dedup): exact repeats of an edge
(either direction) within a fold's chunk are dropped before the fold; the summaries
must be identical to the oracle's. Streams: heavy repetition (edges drawn from a small
pool), the reference's bipartite example stream (every edge 10 times,
BipartitenessCheckExample.java:109-118), ids equal to the table's empty marker (-1),
self-loops, and every fold entry point (host, device, pipelined, window take)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pool_stream(rng, n, pool, idspace):
    a = rng.integers(-idspace, idspace, pool, dtype=np.int64)
    b = rng.integers(-idspace, idspace, pool, dtype=np.int64)
    a[:3] = -1  # the dedup table's empty marker as a real id: never deduplicated, still folded
    b[5] = a[5]  # a self-loop
    k = rng.integers(0, pool, n)
    flip = rng.random(n) < 0.5  # (u, v) and (v, u) are the same pair
    s = np.where(flip, b[k], a[k])
    d = np.where(flip, a[k], b[k])
    return s, d


@pytest.mark.parametrize("mode", ["device", "pipelined", "host", "take"])
def test_dedup_cc_matches_oracle(gs, oracle_mod, mode):
    import torch
    rng = np.random.default_rng(17)
    s, d = _pool_stream(rng, 1 << 17, 3000, 1 << 12)
    ts, td = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    torch.cuda.synchronize()
    B = 1 << 13
    with gs.Summary("cc", capacity_hint=64) as x:
        x.set_batch_dedup(True)
        if mode == "pipelined":
            x.set_pipelining(3)
        if mode == "take":
            x.set_delta_tracking(True)
            rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        for o in range(0, len(s), B):
            if mode == "host":
                x.fold(s[o:o + B], d[o:o + B])
            elif mode == "take":
                x.fold_take(ts[o:], td[o:], B, rec, B, cnt)
            else:
                x.fold_device(ts[o:], td[o:], n=B)
        v, lab = x.labels()
    ov, olab = oracle_mod.cc_labels(s, d)
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_dedup_take_records_replay(gs, oracle_mod):
    """with dedup, a window's records still rebuild the summary (the dropped repeats
    made no structural change)"""
    import torch
    rng = np.random.default_rng(5)
    s, d = _pool_stream(rng, 1 << 16, 2000, 1 << 11)
    ts, td = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    B = 1 << 12
    rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 12) as x, gs.Summary("cc", capacity_hint=1 << 12) as rep:
        x.set_delta_tracking(True)
        x.set_batch_dedup(True)
        for o in range(0, len(s), B):
            x.fold_take(ts[o:], td[o:], B, rec, B, cnt)
            rep.fold_records(rec, x.last_take_word)
            rep.sync()
        v1, l1 = x.labels()
        v2, l2 = rep.labels()
    ov, olab = oracle_mod.cc_labels(s, d)
    assert np.array_equal(v1, ov) and np.array_equal(l1, olab)
    assert np.array_equal(v2, ov) and np.array_equal(l2, olab)


def test_dedup_signed_reference_example_stream(gs, oracle_mod):
    """BipartitenessCheckExample's default stream: (k, 2k+1) ten times each, k = 1..100,
    one window: bipartite; then an odd cycle closed by a repeated same-side pair."""
    import torch
    ks = np.repeat(np.arange(1, 101, dtype=np.int64), 10)
    s, d = ks, 2 * ks + 1
    with gs.Summary("signed", capacity_hint=256) as x:
        x.set_batch_dedup(True)
        x.fold(s, d)
        ok, comp, v, sign = x.colouring()
    tok, tcomp, tv, tsign = oracle_mod.bip_truth(s, d)
    assert ok and tok
    assert np.array_equal(comp, tcomp) and np.array_equal(v, tv) and np.array_equal(sign, tsign)
    # the reference's golden prefix of this stream: components keyed 1, 2, 4, ...
    assert comp.min() == 1 and len(np.unique(comp)) == 51
    # a triangle 1-3-7 repeated: (1,3) and (3,7) exist; (1,7) closes an odd cycle
    s2 = np.concatenate([s, np.full(10, 1, np.int64)])
    d2 = np.concatenate([d, np.full(10, 7, np.int64)])
    with gs.Summary("signed", capacity_hint=256) as x:
        x.set_batch_dedup(True)
        ts, td = torch.from_numpy(s2).cuda(), torch.from_numpy(d2).cuda()
        torch.cuda.synchronize()
        x.fold_device(ts, td, n=len(s2))
        assert x.ok() == oracle_mod.bip_truth(s2, d2)[0]


def test_dedup_rmat_batches_equal_plain(gs, oracle_mod):
    """RMAT-16 in 2^16-edge batches: dedup on equals the oracle (few repeats to drop)."""
    import torch
    n = 1 << 20
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, 16, 0x5EED0026, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 16) as x:
        x.set_batch_dedup(True)
        x.set_pipelining(3)
        for o in range(0, n, 1 << 16):
            x.fold_device(src[o:], dst[o:], n=1 << 16)
        v, lab = x.labels()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)
