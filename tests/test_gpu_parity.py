"""GPU parity: the HIP summary (through the C ABI) against the oracle and the
reference's own vectors. Bit-exact for every integer output."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
I64_MIN = np.iinfo(np.int64).min
I64_MAX = np.iinfo(np.int64).max


def _pins():
    with open(os.path.join(GOLD, "reference_pins.json")) as f:
        return json.load(f)


def _derived():
    with open(os.path.join(GOLD, "derived.json")) as f:
        return json.load(f)


def _cc_string(summary, oracle_mod):
    v, lab = summary.labels()
    return oracle_mod.canonical_cc_string(v, lab)


def _assert_cc_equal(summary, oracle_mod, src, dst):
    v, lab = summary.labels()
    ov, olab = oracle_mod.cc_labels(src, dst)
    assert np.array_equal(v, ov), "vertex sets differ"
    assert np.array_equal(lab, olab), "labels differ at %d vertices" % int((lab != olab).sum())


# ------------------------------------------------------------- reference pins
def test_connected_components_test(gs, oracle_mod):
    p = _pins()["cc_test"]
    s, d = map(np.array, zip(*p["edges"]))
    with gs.Summary("cc", capacity_hint=16) as ds:
        ds.fold(s, d)
        assert oracle_mod.cc_test_parser([_cc_string(ds, oracle_mod)]) == p["expected_lines"]
        assert ds.num_vertices() == 8  # 1,2,3,5,6,7,8,9


def test_bipartiteness_test_bipartite(gs, oracle_mod):
    p = _pins()["bip_test_bipartite"]
    s, d = map(np.array, zip(*p["edges"]))
    with gs.Summary("signed", capacity_hint=16) as c:
        c.fold(s, d)
        assert [oracle_mod.canonical_candidates_string(*c.colouring())] == p["expected"]


def test_bipartiteness_test_non_bipartite(gs, oracle_mod):
    p = _pins()["bip_test_non_bipartite"]
    s, d = map(np.array, zip(*p["edges"]))
    with gs.Summary("signed", capacity_hint=16) as c:
        c.fold(s, d)
        assert not c.ok()
        assert [oracle_mod.canonical_candidates_string(*c.colouring())] == p["expected"]
        # sticky: more edges keep (false,{})
        c.fold(np.array([100]), np.array([101]))
        assert [oracle_mod.canonical_candidates_string(*c.colouring())] == ["(false,{})"]


def test_disjointset_test(gs):
    # DisjointSetTest.java:37-77 on the GPU summary (Integer ids widen to int64)
    p = _pins()["disjointset_test"]
    with gs.Summary("cc", capacity_hint=16) as ds:
        s, d = map(np.array, zip(*p["setup_unions"]))
        ds.fold(s, d)
        assert ds.num_vertices() == p["expected_matches"]
        r1, r2 = ds.find(0), ds.find(1)
        assert r1 != r2
        for i in range(10):
            assert ds.find(i) == (r1 if i % 2 == 0 else r2)
        with gs.Summary("cc", capacity_hint=16) as ds2:
            s, d = map(np.array, zip(*p["merge_unions"]))
            ds2.fold(s, d)
            ds2.combine(ds)  # ds2.merge(ds)
            assert ds2.num_vertices() == p["expected_matches_after_merge"]
            v, lab = ds2.labels()
            assert len(set(lab.tolist())) == p["expected_roots_after_merge"]
        assert ds.find(12345) is None  # find of an unknown vertex -> null


def test_cc_default_stream_per_window(gs, oracle_mod):
    # ConnectedComponentsExample default stream, 1000 ms windows: the cumulative
    # summary after every window (Merger emission) equals the derived golden.
    em = _derived()["cc_default_stream"]["emissions"]
    k = np.arange(1, 101, dtype=np.int64)
    win = (k * 100) // 1000
    with gs.Summary("cc", capacity_hint=256) as ds:
        for wi, w in enumerate(sorted(set(win.tolist()))):
            m = win == w
            ds.fold(k[m], k[m] + 2)
            assert _cc_string(ds, oracle_mod) == em[wi]


def test_bip_default_stream(gs, oracle_mod):
    em = _derived()["bip_default_stream"]["emissions"]
    k = np.repeat(np.arange(1, 101, dtype=np.int64), 10)
    with gs.Summary("signed", capacity_hint=512) as c:
        c.fold(k, 2 * k + 1)
        assert [oracle_mod.canonical_candidates_string(*c.colouring())] == em


# ------------------------------------------------------------- random streams vs oracle
@pytest.mark.parametrize("scramble", [False, True])
@pytest.mark.parametrize("batch", [1, 7, 1000, 1 << 14])
def test_rmat12_batches(gs, oracle_mod, scramble, batch):
    s, d = oracle_mod.rmat_edges(0x5EED0012, 12, 0, 1 << 14, scramble)
    with gs.Summary("cc", capacity_hint=1 << 12) as ds:
        for i in range(0, len(s), batch):
            ds.fold(s[i:i + batch], d[i:i + batch])
        _assert_cc_equal(ds, oracle_mod, s, d)


def test_rmat12_fixture(gs):
    z = np.load(os.path.join(GOLD, "streams.npz"))
    with gs.Summary("cc", capacity_hint=1 << 12) as ds:
        ds.fold(z["rmat12_src"], z["rmat12_dst"])
        v, lab = ds.labels()
        assert np.array_equal(v, z["rmat12_v"]) and np.array_equal(lab, z["rmat12_label"])


def test_er_negative_and_extreme_ids(gs, oracle_mod):
    rng = np.random.default_rng(5)
    pool = np.array([I64_MIN, I64_MIN + 1, -1, 0, 1, I64_MAX - 1, I64_MAX], dtype=np.int64)
    pool = np.concatenate([pool, rng.integers(I64_MIN, I64_MAX, 500, dtype=np.int64)])
    s = rng.choice(pool, 3000)
    d = rng.choice(pool, 3000)
    with gs.Summary("cc", capacity_hint=64) as ds:
        ds.fold(s[:1500], d[:1500])
        ds.fold(s[1500:], d[1500:])
        _assert_cc_equal(ds, oracle_mod, s, d)
        assert ds.find(I64_MIN) in (None, I64_MIN)


def test_empty_and_self_loops(gs, oracle_mod):
    with gs.Summary("cc", capacity_hint=16) as ds:
        ds.fold(np.array([], np.int64), np.array([], np.int64))
        assert ds.num_vertices() == 0
        ds.fold(np.array([3, 3, 4]), np.array([3, 3, 4]))
        assert ds.num_vertices() == 2
        v, lab = ds.labels()
        assert v.tolist() == [3, 4] and lab.tolist() == [3, 4]


def test_table_starts_at_four_slots_per_hinted_vertex(gs):
    """gs_create sizes the table at >= 4 slots per hinted vertex (load <= 1/4: short
    linear-probe clusters, DESIGN.md §3 "Load factor"), never below 1024 slots."""
    for hint, want in ((1, 1024), (1000, 4096), (1 << 20, 1 << 22)):
        with gs.Summary("cc", capacity_hint=hint) as ds:
            assert ds.table_capacity() == want, (hint, ds.table_capacity())


def test_table_growth_from_tiny_hint(gs, oracle_mod):
    s, d = oracle_mod.rmat_edges(99, 16, 0, 1 << 17, True)
    with gs.Summary("cc", capacity_hint=1) as ds:
        for i in range(0, len(s), 1 << 13):
            ds.fold(s[i:i + (1 << 13)], d[i:i + (1 << 13)])
        assert ds.table_capacity() > 1024
        _assert_cc_equal(ds, oracle_mod, s, d)


@pytest.mark.parametrize("depth", [1, 3])
def test_growth_under_pipelined_device_folds(gs, oracle_mod, depth):
    """Capacity tracking from the k_report words (no host sync per fold): device
    folds on 3 lanes from a tiny hint must grow the table in time (a missed bound
    would overflow it: CTR_ERR -> GSError) and stay bit-exact."""
    import torch
    n, B = 1 << 18, 1 << 12
    s = torch.empty(n, dtype=torch.int64, device="cuda")
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_er(s, d, 0, n, 17, 0x5EED00E5, True)  # ER: nearly every endpoint is new early on
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=16) as ds:
        ds.set_pipelining(depth)
        for i in range(0, n, B):
            ds.fold_device(s[i:], d[i:], n=B)
        assert ds.table_capacity() >= 1 << 17
        _assert_cc_equal(ds, oracle_mod, s.cpu().numpy(), d.cpu().numpy())


def test_rmat20_config2_full(gs, oracle_mod):
    # BASELINE config 2: RMAT-20, 16M edges, sparse ids, 1M-edge micro-batches.
    import torch
    n = 1 << 24
    s = torch.empty(n, dtype=torch.int64, device="cuda")
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(s, d, 0, n, 20, 0x5EED0020, True)
    torch.cuda.synchronize()
    hs, hd = s.cpu().numpy(), d.cpu().numpy()
    os_, od = oracle_mod.rmat_edges(0x5EED0020, 20, 0, 1 << 12, True)
    assert np.array_equal(hs[:1 << 12], os_) and np.array_equal(hd[:1 << 12], od)
    with gs.Summary("cc", capacity_hint=1 << 20) as ds:
        for i in range(0, n, 1 << 20):
            ds.fold_device(s[i:], d[i:], n=1 << 20)
        ds.sync()
        _assert_cc_equal(ds, oracle_mod, hs, hd)


@pytest.mark.parametrize("hint", [1 << 18, 64])
def test_pipelined_folds_match_ordered(gs, oracle_mod, hint):
    # gs_set_pipelining(2): consecutive device folds overlap on two lane streams; the
    # labels (and the growth path from a tiny hint) must match the oracle exactly.
    import torch
    n, b = 1 << 20, 1 << 15
    s = torch.empty(n, dtype=torch.int64, device="cuda")
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(s, d, 0, n, 18, 0x5EED0018, True)
    torch.cuda.synchronize()
    hs, hd = s.cpu().numpy(), d.cpu().numpy()
    with gs.Summary("cc", capacity_hint=hint) as ds:
        ds.set_pipelining(2)
        for i in range(0, n, b):
            ds.fold_device(s[i:], d[i:], n=b)
            if i == n // 2:
                assert ds.num_vertices() > 0  # a read in the middle joins the lanes
        _assert_cc_equal(ds, oracle_mod, hs, hd)
        ds.reset()
        for i in range(0, n // 4, b):
            ds.fold_device(s[i:], d[i:], n=b)
        _assert_cc_equal(ds, oracle_mod, hs[:n // 4], hd[:n // 4])


def test_pipelined_signed_folds(gs, oracle_mod):
    s, d = oracle_mod.rmat_edges(0x5EED0B1C, 14, 0, 1 << 16, True)
    import torch
    ts = torch.from_numpy(s).cuda()
    td = torch.from_numpy(d).cuda()
    with gs.Summary("signed", capacity_hint=1 << 14) as a, gs.Summary("signed", capacity_hint=1 << 14) as b:
        a.set_pipelining(2)
        for i in range(0, len(s), 1 << 12):
            a.fold_device(ts[i:], td[i:], n=1 << 12)
            b.fold_device(ts[i:], td[i:], n=1 << 12)
        ca, cb = a.colouring(), b.colouring()
        assert ca[0] == cb[0]
        assert all(np.array_equal(x, y) for x, y in zip(ca[1:], cb[1:]))


@pytest.mark.parametrize("kind,nparts", [("cc", 1), ("cc", 3), ("cc", 8), ("signed", 5)])
def test_export_parts_partition_the_label_pass(gs, oracle_mod, kind, nparts):
    """gs_export_labels_part_device: the parts are disjoint and together equal the
    whole export (incl. the reserved INT64_MIN / INT64_MIN + 1 slots at the end)."""
    import torch
    if kind == "cc":
        s, d = oracle_mod.rmat_edges(0x5EED0026, 13, 0, 1 << 16, True)
        s = np.concatenate([s, np.array([np.iinfo(np.int64).min, 7], np.int64)])
        d = np.concatenate([d, np.array([np.iinfo(np.int64).min + 1, np.iinfo(np.int64).min], np.int64)])
    else:
        s, d = oracle_mod.bip_edges(0x5EED0B1B, 11, 0, 1 << 15)
    with gs.Summary(kind, capacity_hint=1 << 14) as x:
        x.fold(s, d)
        n = x.num_vertices()
        v = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        lab = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        par = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
        got = x.export_labels_device(v, lab, par)
        whole = sorted(zip(v[:got].tolist(), lab[:got].tolist(), par[:got].tolist()))
        parts = []
        for p in range(nparts):
            k = x.export_labels_part_device(p, nparts, v, lab, par)
            parts += list(zip(v[:k].tolist(), lab[:k].tolist(), par[:k].tolist()))
        assert len(parts) == got == n
        assert sorted(parts) == whole


# ------------------------------------------------------------- combine / serialize / delta
def test_combine_equals_whole(gs, oracle_mod):
    s, d = oracle_mod.rmat_edges(3, 14, 0, 1 << 16, True)
    h = len(s) // 2
    with gs.Summary("cc", capacity_hint=1 << 14) as a, gs.Summary("cc", capacity_hint=1 << 10) as b:
        a.fold(s[:h], d[:h])
        b.fold(s[h:], d[h:])
        a.combine(b)  # CombineCC: merge
        _assert_cc_equal(a, oracle_mod, s, d)


def test_serialize_roundtrip(gs, oracle_mod):
    s, d = oracle_mod.rmat_edges(4, 12, 0, 1 << 13, True)
    with gs.Summary("cc", capacity_hint=1 << 12) as a, gs.Summary("cc", capacity_hint=4) as b:
        a.fold(s, d)
        img = a.serialize()
        b.deserialize(img)
        va, la = a.labels()
        vb, lb = b.labels()
        assert np.array_equal(va, vb) and np.array_equal(la, lb)


def test_delta_exchange_reproduces_union(gs, oracle_mod):
    # Two replicas fold disjoint halves of each batch and fold each other's delta
    # records: afterwards both equal the whole stream (the multi-GPU combine step).
    import torch
    s, d = oracle_mod.rmat_edges(5, 14, 0, 1 << 16, True)
    reps = [gs.Summary("cc", capacity_hint=1 << 13) for _ in range(2)]
    for r in reps:
        r.set_delta_tracking(True)
    B = 1 << 12
    cap = 3 * B
    recs = [torch.empty((cap, 3), dtype=torch.int64, device="cuda") for _ in range(2)]
    cnts = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    total = 0
    for i in range(0, len(s), 2 * B):
        reps[0].fold(s[i:i + B], d[i:i + B])
        reps[1].fold(s[i + B:i + 2 * B], d[i + B:i + 2 * B])
        for k in range(2):
            reps[k].take_delta_records(recs[k], cap, cnts[k])
            reps[k].sync()
        ns = [int(c.item()) for c in cnts]
        assert max(ns) <= cap
        total += sum(ns)
        for k in range(2):
            reps[1 - k].fold_records(recs[k], ns[k], track=False)
            reps[1 - k].sync()  # rec is reused by the next take
    for r in reps:
        _assert_cc_equal(r, oracle_mod, s, d)
        r.close()
    # hooked new vertices are filtered: far fewer records than 2 per edge + hooks
    assert total < len(s)


def _stage_and_gather(gs, reps, width):
    """Every replica stages its delta (gs_delta_stage); the buffers are concatenated
    the way the data all-gather lays them out: world blocks of max-count rows."""
    import torch
    world = len(reps)
    cap = reps[0].delta_capacity()
    sends = [torch.empty((cap, width), dtype=torch.int64, device="cuda") for _ in range(world)]
    counts = torch.zeros(world, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    for r in range(world):
        reps[r].delta_stage(sends[r], cap, counts[r:r + 1], width)
        reps[r].sync()
    live = [int(c) & ((1 << 62) - 1) for c in counts.tolist()]
    rows = max(1, max(live))
    recv = torch.cat([x[:rows] for x in sends]).contiguous()
    return recv, counts, rows, live


@pytest.mark.parametrize("width", [2, 3])
def test_delta_stage_and_exchange_fold(gs, oracle_mod, width):
    # every replica stages its whole delta; folding the gathered buffer (live rows of
    # each block from the count words) reproduces the union on every replica
    s, d = oracle_mod.rmat_edges(6, 13, 0, 1 << 15, True)
    world, B = 3, 1 << 11
    reps = [gs.Summary("cc", capacity_hint=1 << 12) for _ in range(world)]
    for r in reps:
        r.set_delta_tracking(True)
    assert reps[0].delta_capacity() >= 1 << 22
    padded = 0
    for i in range(0, len(s), world * B):
        for r in range(world):
            lo = i + r * B
            reps[r].fold(s[lo:lo + B], d[lo:lo + B])
        recv, counts, rows, live = _stage_and_gather(gs, reps, width)
        assert max(live) <= B  # at most one record per folded edge
        padded += world * rows - sum(live)
        for r in range(world):
            reps[r].fold_exchange(recv, counts, world, rows, r, width)
    for r in reps:
        _assert_cc_equal(r, oracle_mod, s, d)
        r.close()


@pytest.mark.parametrize("skip", [-1, 7])
def test_exchange_fold_grows_table_from_remote_rows(gs, oracle_mod, skip):
    # A replica that folds nothing itself receives every vertex through exchange
    # folds; its tiny table must grow in time: labels equal the oracle's.
    # skip = -1 folds every block; skip = 7 (no such rank) must not drop a block.
    s, d = oracle_mod.rmat_edges(6, 12, 0, 1 << 14, True)
    world, B = 3, 1 << 10
    senders = [gs.Summary("cc", capacity_hint=1 << 13) for _ in range(world)]
    sink = gs.Summary("cc", capacity_hint=64)
    for r in senders:
        r.set_delta_tracking(True)
    for i in range(0, len(s), world * B):
        for r in range(world):
            lo = i + r * B
            senders[r].fold(s[lo:lo + B], d[lo:lo + B])
        recv, counts, rows, live = _stage_and_gather(gs, senders, 3)
        sink.fold_exchange(recv, counts, world, rows, skip, 3)
    _assert_cc_equal(sink, oracle_mod, s, d)
    for r in senders + [sink]:
        r.close()


def test_exchange_count_word_carries_signed_failure(gs, oracle_mod):
    """a rank whose replica finds an odd cycle among vertices it
    already connected produces NO record for that edge; the count word's failure bit
    must carry the verdict to every other replica."""
    import torch
    with gs.Summary("signed", capacity_hint=64) as a, gs.Summary("signed", capacity_hint=64) as b:
        for x in (a, b):
            x.set_delta_tracking(True)
        a.fold(np.array([1, 2]), np.array([2, 3]))  # path 1-2-3
        b.fold(np.array([10]), np.array([11]))
        recv, counts, rows, live = _stage_and_gather(gs, [a, b], 3)
        for r, x in enumerate((a, b)):
            x.fold_exchange(recv, counts, 2, rows, r, 3)
        a.fold(np.array([1]), np.array([3]))  # odd cycle inside a's replica: a hook-free failure
        assert not a.ok() and b.ok()
        recv, counts, rows, live = _stage_and_gather(gs, [a, b], 3)
        assert live[0] == 0 and (int(counts[0]) >> 62) & 1 == 1
        b.fold_exchange(recv, counts, 2, rows, 1, 3)
        assert not b.ok()
        assert [oracle_mod.canonical_candidates_string(*b.colouring())] == ["(false,{})"]


def test_delta_records_skip_padding(gs, oracle_mod):
    import torch
    rec = torch.tensor([[1, 2, 0], [3, 4, 0x80], [5, 6, 0], [7, 7, 0x80]], dtype=torch.int64, device="cuda")
    with gs.Summary("cc", capacity_hint=64) as a:
        a.fold_records(rec, 4)
        v, lab = a.labels()
        assert v.tolist() == [1, 2, 5, 6] and lab.tolist() == [1, 1, 5, 5]


# ------------------------------------------------------------- bipartiteness
def test_bip_random_vs_truth(gs, oracle_mod):
    rng = np.random.default_rng(6)
    for trial in range(30):
        n = int(rng.integers(2, 200))
        m = int(rng.integers(1, 400))
        s = rng.integers(-n, n, m)
        d = rng.integers(-n, n, m)
        with gs.Summary("signed", capacity_hint=64) as c:
            for i in range(0, m, 37):
                c.fold(s[i:i + 37], d[i:i + 37])
            truth = oracle_mod.canonical_candidates_string(*oracle_mod.bip_truth(s, d))
            assert oracle_mod.canonical_candidates_string(*c.colouring()) == truth


def test_bip_exact_regime_matches_reference_quirk_oracle(gs, oracle_mod):
    # first-appearance ids, one window, p = 1: the reference's own Candidates
    # output (quirk-exact restatement) equals the GPU output string.
    rng = np.random.default_rng(7)
    for trial in range(40):
        n = int(rng.integers(2, 40))
        m = int(rng.integers(1, 60))
        raw_s = rng.integers(0, n, m)
        raw_d = rng.integers(0, n, m)
        ids = {}
        for a, b in zip(raw_s.tolist(), raw_d.tolist()):
            for x in (a, b):
                ids.setdefault(x, len(ids) + 1)
        s = np.array([ids[x] for x in raw_s.tolist()], np.int64)
        d = np.array([ids[x] for x in raw_d.tolist()], np.int64)
        with gs.Summary("signed", capacity_hint=64) as c:
            c.fold(s, d)
            assert [oracle_mod.canonical_candidates_string(*c.colouring())] == oracle_mod.bip_dataflow(s, d)


def test_bip_config4_injected_odd_cycles(gs, oracle_mod):
    import torch
    E = 1 << 20
    inject = [E // 8, E // 4, E // 2, 3 * E // 4]
    s = torch.empty(E, dtype=torch.int64, device="cuda")
    d = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_bip(s, d, 0, E, 15, 0x5EED0B1B, inject)
    torch.cuda.synchronize()
    hs, hd = s.cpu().numpy(), d.cpu().numpy()
    os_, od = oracle_mod.bip_edges(0x5EED0B1B, 15, 0, E, inject)
    assert np.array_equal(hs, os_) and np.array_equal(hd, od)
    first = oracle_mod.bip_first_failure(hs, hd)
    B = 1 << 16
    with gs.Summary("signed", capacity_hint=1 << 16) as c:
        for i in range(0, E, B):
            c.fold_device(s[i:], d[i:], n=B)
            expect_ok = first < 0 or first >= i + B
            assert c.ok() == expect_ok, (i, first)
    # clean variant stays bipartite, colouring equals truth
    gs.gen_bip(s, d, 0, E, 15, 0x5EED0B1B, [])
    torch.cuda.synchronize()
    with gs.Summary("signed", capacity_hint=1 << 16) as c:
        c.fold_device(s, d, n=E)
        ok, comp, v, sign = c.colouring()
        tok, tcomp, tv, tsign = oracle_mod.bip_truth(s.cpu().numpy(), d.cpu().numpy())
        assert ok and tok
        assert np.array_equal(comp, tcomp) and np.array_equal(v, tv) and np.array_equal(sign, tsign)


def test_bip_combine_and_serialize(gs, oracle_mod):
    s, d = oracle_mod.bip_edges(9, 8, 0, 2000, [])
    with gs.Summary("signed", capacity_hint=512) as a, gs.Summary("signed", capacity_hint=512) as b:
        a.fold(s[:1000], d[:1000])
        b.fold(s[1000:], d[1000:])
        a.combine(b)
        truth = oracle_mod.canonical_candidates_string(*oracle_mod.bip_truth(s, d))
        assert oracle_mod.canonical_candidates_string(*a.colouring()) == truth
        img = a.serialize()
        b.deserialize(img)
        assert oracle_mod.canonical_candidates_string(*b.colouring()) == truth
        b.fold(np.array([0]), np.array([2]))  # same side, connected? may fail
        ok_truth = oracle_mod.bip_truth(np.append(s, 0), np.append(d, 2))[0]
        assert b.ok() == ok_truth


# ------------------------------------------------------------- generators
def test_gpu_generators_match_oracle(gs, oracle_mod):
    import torch
    n = 1 << 14
    s = torch.empty(n, dtype=torch.int64, device="cuda")
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    for scale, seed, start in ((26, 0x5EED0026, (1 << 30) - n), (20, 0x5EED0020, 12345)):
        for scr in (True, False):
            gs.gen_rmat(s, d, start, n, scale, seed, scr)
            torch.cuda.synchronize()
            os_, od = oracle_mod.rmat_edges(seed, scale, start, n, scr)
            assert np.array_equal(s.cpu().numpy(), os_) and np.array_equal(d.cpu().numpy(), od)
    gs.gen_er(s, d, 777, n, 22, 0x5EED00E5, True)
    torch.cuda.synchronize()
    os_, od = oracle_mod.er_edges(0x5EED00E5, 22, 777, n, True)
    assert np.array_equal(s.cpu().numpy(), os_) and np.array_equal(d.cpu().numpy(), od)


# ------------------------------------------------------------- vertex list / resets / batched find
@pytest.mark.parametrize("hint", [1 << 20, 1 << 10])
def test_vertex_list_reset_and_export(gs, oracle_mod, hint):
    """Sparse tables reset and export over the vertex list (O(vertices)); dense ones
    scan the table. Both must leave exactly the initial table / every vertex:
    alternate streams through one handle (a pooled window partial) and compare."""
    with gs.Summary("cc", capacity_hint=hint) as ds:
        for seed in range(4):
            s, d = oracle_mod.rmat_edges(100 + seed, 12 + seed % 2, 0, 1 << (12 + seed), True)
            s = np.concatenate([s, np.array([I64_MIN, 5], np.int64)])
            d = np.concatenate([d, np.array([I64_MIN, I64_MIN], np.int64)])
            ds.reset()
            for i in range(0, len(s), 1000):
                ds.fold(s[i:i + 1000], d[i:i + 1000])
            _assert_cc_equal(ds, oracle_mod, s, d)
            assert ds.find(I64_MIN) == I64_MIN and ds.find(5) == I64_MIN
        ds.reset()
        assert ds.num_vertices() == 0 and ds.find(5) is None
        v, lab = ds.labels()
        assert len(v) == 0


def test_small_folds_rotate_shards(gs, oracle_mod):
    """Many one-block folds: the rotating first shard spreads the vertex list over
    all 64 shards, so no shard overflows (the list stays usable: counters bit 1 off)."""
    s, d = oracle_mod.er_edges(0x5EED00E5, 16, 0, 1 << 15, True)
    with gs.Summary("cc", capacity_hint=1 << 15) as ds:
        for i in range(0, len(s), 200):
            ds.fold(s[i:i + 200], d[i:i + 200])
        assert (ds.counters()["ovf"] & 2) == 0
        _assert_cc_equal(ds, oracle_mod, s, d)


def test_find_labels_device(gs, oracle_mod):
    import torch
    s, d = oracle_mod.rmat_edges(0x5EED0026, 14, 0, 1 << 16, True)
    ov, olab = oracle_mod.cc_labels(s, d)
    with gs.Summary("cc", capacity_hint=1 << 14) as ds:
        ds.fold(s, d)
        q = np.concatenate([ov, np.array([123456789, I64_MIN], np.int64)])
        tq = torch.from_numpy(q).cuda()
        lab = torch.empty_like(tq)
        found = torch.empty(len(q), dtype=torch.uint8, device="cuda")
        ds.find_labels_device(tq, lab, found)
        ds.sync()
        assert np.array_equal(lab.cpu().numpy()[:len(ov)], olab)
        assert found.cpu().numpy().tolist() == [1] * len(ov) + [0, 0]
        assert int(lab[-2]) == 123456789


def test_capacity_sync_then_near_limit_fold_does_not_stall(gs, oracle_mod):
    """after a synchronising capacity check, edges left unclaimed
    by any report must not make later checks spin their 200 ms wait."""
    import torch
    n, B = 1 << 18, 1 << 12
    s = torch.empty(n, dtype=torch.int64, device="cuda")
    d = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_er(s, d, 0, n, 17, 0x5EED00E5, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=16) as ds:
        ds.set_pipelining(3)
        for i in range(0, n, B):
            ds.fold_device(s[i:], d[i:], n=B)
        st = ds.capacity_stats()
        assert st["syncs"] >= 1
        # no wait may last the full 200 ms budget
        assert st["wait_ms"] < 150 * max(1, st["waits"]), st
        _assert_cc_equal(ds, oracle_mod, s.cpu().numpy(), d.cpu().numpy())


def test_delta_list_full_error_leaves_capacity_tracking_intact(gs, oracle_mod):
    """A tracked fold refused for a full delta list must not charge its edges to the
    capacity bound (they are never folded, so no report would ever claim them and
    every later capacity check would wait out its 200 ms timeout). Fold until the
    list refuses, take, go on: no fold + sync may take anywhere near 200 ms, and the
    labels equal the oracle."""
    import time
    import torch
    n, B = 1 << 23, 1 << 18  # the delta list holds >= 2^22 folded edges (kMaxChunk)
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_er(src, dst, 0, n, 17, 0x5EED00E5, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 17) as s:
        s.set_delta_tracking(True)
        cap = s.delta_capacity()
        rec = torch.empty((cap, 3), dtype=torch.int64, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
        refused, worst, o = 0, 0.0, 0
        while o < n:
            t0 = time.perf_counter()
            try:
                s.fold_device(src[o:], dst[o:], n=B)
                s.sync()
                o += B
            except gs.GSError:
                refused += 1
                s.take_delta_records(rec, cap, cnt)
                s.sync()
            worst = max(worst, time.perf_counter() - t0)
        assert refused > 0, "the delta list never filled: the test does not exercise the refusal"
        assert worst < 0.1, "a fold + sync took %.3f s (capacity wait)" % worst
        v, lab = s.labels()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_digest_matches_restatement_and_is_order_free(gs, oracle_mod):
    """gs_digest (the N > 1 bench line's label self-check) equals the
    checker's restatement over the oracle's labels, is independent of fold order,
    windowing and pipelining, differs when one edge is missing, and is GS_DIGEST_FAILED for
    a signed summary whose verdict failed."""
    s, d = oracle_mod.rmat_edges(0x5EED0020, 14, 0, 1 << 16, True)
    ov, olab = oracle_mod.cc_labels(s, d)
    want = oracle_mod.label_digest(ov, olab)
    rng = np.random.default_rng(5)
    perm = rng.permutation(len(s))
    digests = []
    for order, chunk, pipe in ((None, 1 << 16, 1), (perm, 1 << 12, 3), (perm[::-1].copy(), 777, 2)):
        ss, dd = (s, d) if order is None else (s[order], d[order])
        with gs.Summary("cc", capacity_hint=1 << 12) as c:
            c.set_pipelining(pipe)
            for o in range(0, len(ss), chunk):
                c.fold(ss[o:o + chunk], dd[o:o + chunk])
            digests.append(c.digest())
    assert digests == [want] * 3
    with gs.Summary("cc", capacity_hint=1 << 12) as c:
        c.fold(s[1:], d[1:])
        v2, l2 = oracle_mod.cc_labels(s[1:], d[1:])
        assert c.digest() == oracle_mod.label_digest(v2, l2)
        if not (np.array_equal(v2, ov) and np.array_equal(l2, olab)):
            assert c.digest() != want
    bs, bd = oracle_mod.bip_edges(0x5EED0B1B, 10, 0, 3000)
    ok, comp, v, sign = oracle_mod.bip_truth(bs, bd)
    with gs.Summary("signed", capacity_hint=1 << 11) as c:
        c.fold(bs, bd)
        assert ok and c.ok()
        # parity(v) xor parity(label) = 1 - sign
        assert c.digest() == oracle_mod.label_digest(v, comp, 1 - np.asarray(sign, np.int64))
        c.fold(np.array([bs[0]], np.int64), np.array([bd[0]], np.int64))  # same edge again: still bipartite
        assert c.ok()
        # an odd cycle: a vertex and its component's minimum, required on the sides they are not on
        i = int(np.nonzero(np.asarray(v) != np.asarray(comp))[0][0])
        w = np.array([1 if sign[i] else 0], np.uint8)
        c.fold_parity(np.array([v[i]], np.int64), np.array([comp[i]], np.int64), w)
        assert not c.ok()
        assert c.digest() == gs.DIGEST_FAILED
