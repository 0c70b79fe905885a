"""The latency path's fused window (gs_fold_take_device: fold + delta take + completion in
one launch, BASELINE config 5) against the oracle and against the separate
fold / take / sync sequence. Reference: per-window PartialAgg.fold then CombineCC and
the Merger (S/SummaryBulkAggregation.java:109-130, S/SummaryAggregation.java:107-119)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _labels_equal(a, b):
    v1, l1 = a.labels()
    v2, l2 = b.labels()
    return np.array_equal(v1, v2) and np.array_equal(l1, l2)


@pytest.mark.parametrize("logn,logb", [(14, 10), (17, 12)])
def test_fused_window_take_matches_oracle_and_replays(gs, oracle_mod, logn, logb):
    """ER windows through fold_take: labels oracle-exact after every checkpoint; the
    taken records alone rebuild the summary; host count == device count <= window."""
    import torch
    E, B = 1 << (logn + 3), 1 << logb
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_er(src, dst, 0, E, logn, 0x5EED00E5, True)
    torch.cuda.synchronize()
    rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    ps, pd = src.data_ptr(), dst.data_ptr()
    with gs.Summary("cc", capacity_hint=1 << logn) as s, gs.Summary("cc", capacity_hint=1 << logn) as rep:
        s.set_delta_tracking(True)
        total = 0
        for w in range(E // B):
            o = w * B
            k = s.fold_take(ps + 8 * o, pd + 8 * o, B, rec, B, cnt)
            assert k == int(cnt.item()) and 0 <= k <= B
            total += k
            rep.fold_records(rec, k)
            rep.sync()  # rec is reused by the next take
            if w + 1 in (1, 2, 7, E // B):
                ov, olab = oracle_mod.cc_labels(hs[:o + B], hd[:o + B])
                v, lab = s.labels()
                assert np.array_equal(v, ov) and np.array_equal(lab, olab), "oracle differs at window %d" % (w + 1)
                assert _labels_equal(s, rep), "replay differs at window %d" % (w + 1)
        # records >= component merges + vertices (every vertex is named by some record)
        assert total >= len(np.unique(np.concatenate([hs, hd]))) - len(set(olab.tolist()))


def test_fused_window_take_self_loops_and_growth(gs, oracle_mod):
    """A 1-vertex capacity hint (the table grows inside the fused path's capacity check),
    self-loops and duplicate edges: still oracle-exact and replayable."""
    import torch
    rng = np.random.default_rng(7)
    n, B = 1 << 14, 1 << 10
    hs = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    hd = hs.copy()
    m = rng.random(n) < 0.7
    hd[m] = rng.choice(hs, int(m.sum()))  # 30 % self-loops, repeated ids
    src = torch.from_numpy(hs).cuda()
    dst = torch.from_numpy(hd).cuda()
    rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    with gs.Summary("cc", capacity_hint=1) as s, gs.Summary("cc", capacity_hint=1) as rep:
        s.set_delta_tracking(True)
        for o in range(0, n, B):
            k = s.fold_take(src[o:], dst[o:], B, rec, B, cnt)
            rep.fold_records(rec, k)
            rep.sync()  # rec is reused by the next take
        ov, olab = oracle_mod.cc_labels(hs, hd)
        v, lab = s.labels()
        assert np.array_equal(v, ov) and np.array_equal(lab, olab)
        assert _labels_equal(s, rep)


def test_fused_window_take_signed_verdict(gs, oracle_mod):
    """Signed kind: the parity rides in the records (w), the verdict flips in the truth's
    window, and after failure the fused launch still completes (every block reaches its
    ticket) with no records. The count word carries the verdict (| FAIL_BIT), so a
    replica that replays every window -- before AND after the flip -- holds the same
    verdict and, while bipartite, the same colouring (Candidates.java:79-81)."""
    import torch
    logside, E, B = 12, 1 << 15, 1 << 11
    inject = [E // 4, E // 2]
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, E, logside, 0x5EED0B1B, inject)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    first = oracle_mod.bip_first_failure(hs, hd)
    assert first >= 0
    rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    with gs.Summary("signed", capacity_hint=1 << 13) as c, gs.Summary("signed", capacity_hint=1 << 13) as rep:
        c.set_delta_tracking(True)
        for o in range(0, E, B):
            k = c.fold_take(src[o:], dst[o:], B, rec, B, cnt)
            word = c.last_take_word
            failed_now = first < o + B
            assert bool(word & gs.FAIL_BIT) == failed_now, (o, first, word)
            assert int(cnt.item()) == word  # the device count word is the same word
            if o >= first + B:
                assert k == 0  # a failed verdict is final: nothing folds, nothing recorded
            rep.fold_records(rec, word)
            rep.sync()  # rec is reused by the next take
            assert c.ok() == (not failed_now), (o, first)
            assert rep.ok() == c.ok(), (o, first)
            if o + B in (B, 4 * B):
                ok, comp, v, sign = rep.colouring()
                tok, tcomp, tv, tsign = oracle_mod.bip_truth(hs[:o + B], hd[:o + B])
                assert ok and tok and np.array_equal(v, tv) and np.array_equal(comp, tcomp) and \
                    np.array_equal(sign, tsign)


def test_signed_take_word_general_path_and_device_replay(gs, oracle_mod):
    """The general (unfused) take path -- records pending from an untaken tracked fold --
    and gs_take_delta_records carry the verdict bit too; a device-side replay
    (fold_records_counted: the count word read on the device) reproduces summary and
    verdict with no host round trip."""
    import torch
    logside, E, B = 11, 1 << 14, 1 << 10
    inject = [E // 2 + 17]
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, E, logside, 0x5EED0B1B, inject)
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    first = oracle_mod.bip_first_failure(hs, hd)
    assert first >= 0
    cap = 2 * B
    rec = torch.empty((cap, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    with gs.Summary("signed", capacity_hint=1 << 12) as c, gs.Summary("signed", capacity_hint=1 << 12) as rep, \
            gs.Summary("signed", capacity_hint=1 << 12) as rep2:
        c.set_delta_tracking(True)
        for o in range(0, E, 2 * B):
            c.fold_device(src[o:], dst[o:], n=B)  # tracked, not taken: the next take is general
            c.sync()
            k = c.fold_take(src[o + B:], dst[o + B:], B, rec, cap, cnt)
            word = c.last_take_word
            assert bool(word & gs.FAIL_BIT) == (first < o + 2 * B), (o, first)
            rep.fold_records(rec, word)
            rep2.fold_records_counted(rec, cap, cnt)
            rep.sync()
            rep2.sync()
            assert rep.ok() == c.ok() == rep2.ok() == (first >= o + 2 * B)
            assert k <= cap
        # gs_take_delta_records: the same word on the device
        c.fold_device(src[:B], dst[:B], n=B)
        c.take_delta_records(rec, cap, cnt)
        c.sync()
        assert int(cnt.item()) & gs.FAIL_BIT
    # CC summaries never carry the bit; a counted replay of a CC take equals the summary
    with gs.Summary("cc", capacity_hint=1 << 12) as c, gs.Summary("cc", capacity_hint=1 << 12) as rep:
        c.set_delta_tracking(True)
        for o in range(0, E, B):
            c.fold_take(src[o:], dst[o:], B, rec, cap, cnt)
            assert c.last_take_word & gs.FAIL_BIT == 0
            rep.fold_records_counted(rec, cap, cnt)
            rep.sync()
        assert _labels_equal(c, rep)
        ov, olab = oracle_mod.cc_labels(hs, hd)
        v, lab = rep.labels()
        assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_fused_window_take_truncates_and_counts(gs):
    """cap below the window's records: only cap rows written, the count says how many."""
    import torch
    n = 1 << 12
    hs = np.arange(0, 2 * n, 2, dtype=np.int64)
    hd = hs + 1  # n disjoint edges: n hook records
    src = torch.from_numpy(hs).cuda()
    dst = torch.from_numpy(hd).cuda()
    cap = 100
    rec = torch.full((cap + 8, 3), -7, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    with gs.Summary("cc", capacity_hint=1 << 14) as s:
        s.set_delta_tracking(True)
        k = s.fold_take(src, dst, n, rec, cap, cnt)
        assert k == n and int(cnt.item()) == n
        r = rec.cpu().numpy()
        assert (r[cap:] == -7).all()  # nothing past cap
        got = {(int(a), int(b)) for a, b, _ in r[:cap]}
        assert len(got) == cap and all(b == a - 1 or a == b - 1 for a, b in got)


def test_fused_window_take_includes_pending_records(gs, oracle_mod):
    """Records of an earlier tracked fold that nobody took belong to the next take
    (general path); the following window is fused again."""
    import torch
    rng = np.random.default_rng(3)
    hs = rng.integers(0, 1 << 12, 3 << 10, dtype=np.int64)
    hd = rng.integers(0, 1 << 12, 3 << 10, dtype=np.int64)
    src = torch.from_numpy(hs).cuda()
    dst = torch.from_numpy(hd).cuda()
    B = 1 << 10
    rec = torch.empty((2 * B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    with gs.Summary("cc", capacity_hint=1 << 13) as s, gs.Summary("cc", capacity_hint=1 << 13) as rep:
        s.set_delta_tracking(True)
        s.fold_device(src[:B], dst[:B], n=B)  # tracked, not taken
        k = s.fold_take(src[B:], dst[B:], B, rec, 2 * B, cnt)
        rep.fold_records(rec, k)
        rep.sync()  # rec is reused by the next take
        k = s.fold_take(src[2 * B:], dst[2 * B:], B, rec, 2 * B, cnt)
        rep.fold_records(rec, k)
        rep.sync()  # rec is reused by the next take
        ov, olab = oracle_mod.cc_labels(hs, hd)
        v, lab = rep.labels()
        assert np.array_equal(v, ov) and np.array_equal(lab, olab)
        assert _labels_equal(s, rep)


@pytest.mark.parametrize("kind", ["cc", "signed"])
def test_window_server_equals_fused_launch(gs, oracle_mod, kind):
    """The resident window server (gs_set_window_server) gives the same windows as the
    fused launch: the same count words (rows | FAIL_BIT) and record sets, replays to the
    same summary, oracle-exact; reads mid-stream stop it and the next window restarts it;
    an idle pause longer than its timeout makes it leave on its own and come back; a tiny
    capacity hint makes the table grow between windows (the server is stopped for it)."""
    import time
    import torch
    E, B = 1 << 18, 1 << 14
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    if kind == "cc":
        gs.gen_er(src, dst, 0, E, 15, 0x5EED00E5, True)
    else:
        gs.gen_bip(src, dst, 0, E, 13, 0x5EED0B1B, [E // 2 + 5])
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    recs = [torch.empty((B, 3), dtype=torch.int64, device="cuda") for _ in range(2)]
    cnts = [torch.zeros(1, dtype=torch.int64, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    with gs.Summary(kind, capacity_hint=1) as srv, gs.Summary(kind, capacity_hint=1 << 16) as ref, \
            gs.Summary(kind, capacity_hint=1 << 16) as rep:
        srv.set_delta_tracking(True)
        ref.set_delta_tracking(True)
        srv.set_window_server(True)
        for w in range(E // B):
            o = w * B
            k1 = srv.fold_take(src[o:], dst[o:], B, recs[0], B, cnts[0])
            k2 = ref.fold_take(src[o:], dst[o:], B, recs[1], B, cnts[1])
            # the verdict bit agrees; the row counts may differ by a self-loop record (which
            # thread inserts a vertex seen twice in one window is a race), the summaries not
            assert (srv.last_take_word ^ ref.last_take_word) & gs.FAIL_BIT == 0, w
            assert int(cnts[0].item()) == srv.last_take_word and k1 <= B and k2 <= B
            rep.fold_records(recs[0], srv.last_take_word)
            rep.sync()
            if w == 3:
                srv.labels()  # any other call stops the server; the next window restarts it
            if w == 6:
                time.sleep(0.6)  # longer than the idle timeout: the server leaves by itself
        st = srv.window_server_stats()
        assert st["windows"] >= E // B - 2 and st["launches"] >= 3, st
        if kind == "cc":
            ov, olab = oracle_mod.cc_labels(hs, hd)
            for s in (srv, ref, rep):
                v, lab = s.labels()
                assert np.array_equal(v, ov) and np.array_equal(lab, olab)
        else:
            tok = oracle_mod.bip_truth(hs, hd)[0]
            assert srv.ok() == ref.ok() == rep.ok() == tok


@pytest.mark.parametrize("how", ["stream", "event"])
def test_window_server_stops_for_a_wait(gs, oracle_mod, how):
    """a wait (gs_wait_stream / gs_wait_event) must order the next window
    behind the producer even while the resident server runs. Each window is copied into
    ONE reused buffer on a torch stream behind a GPU sleep and ordered by a wait only (no
    host synchronisation): the wait stops the server, and the window starts a new server
    launch queued behind it. Without that, the running server would fold the buffer
    before (or while) the producer writes it."""
    import torch
    E, B = 1 << 16, 1 << 12
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_er(src, dst, 0, E, 14, 0x5EED00E5, True)
    torch.cuda.synchronize()
    bs = torch.zeros(B, dtype=torch.int64, device="cuda")
    bd = torch.zeros(B, dtype=torch.int64, device="cuda")
    rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    prod = torch.cuda.Stream()
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 14) as s:
        s.set_delta_tracking(True)
        s.set_window_server(True)
        s.fold_take(src, dst, 1, rec, B, cnt)  # the server is running now
        for w in range(E // B):
            o = w * B
            with torch.cuda.stream(prod):
                torch.cuda._sleep(300000)  # the writer is still busy when the window is posted
                bs.copy_(src[o:o + B])
                bd.copy_(dst[o:o + B])
                ev = torch.cuda.Event()
                ev.record(prod)
            if how == "stream":
                s.wait_stream(prod)
            else:
                s.wait_event(ev)
            s.fold_take(bs, bd, B, rec, B, cnt)  # returns when the window is complete
        st = s.window_server_stats()
        assert st["launches"] >= E // B, st  # every wait stopped the server
        v, lab = s.labels()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["cc", "signed"])
def test_window_server_mixed_window_sizes(gs, oracle_mod, kind):
    """The server's take tails over every window shape in one session: one block (64
    edges: the one-drain tail), 2 and 16 blocks (one ticket level), 64 blocks (two
    levels). CC windows carry rows and inserts through the tickets and keep the session's
    vertex count (CTR_SRV_NV), which the host uses for capacity: a tiny hint makes the
    table grow between windows, so a wrong count would overflow it. Every window's count
    word equals its rows, the replay of all windows equals the summary, and both equal
    the oracle."""
    import torch
    sizes = [64, 300, 4096, 1 << 14]
    E = 24 * sum(sizes)
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    if kind == "cc":
        gs.gen_er(src, dst, 0, E, 16, 0x5EED00E7, True)
    else:
        gs.gen_bip(src, dst, 0, E, 14, 0x5EED0B1D, [E // 3])  # an odd cycle a third of the way in
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    cap = max(sizes) + 16
    rec = torch.empty((cap, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    with gs.Summary(kind, capacity_hint=1) as srv, gs.Summary(kind, capacity_hint=1 << 16) as rep:
        srv.set_delta_tracking(True)
        srv.set_window_server(True)
        o, w = 0, 0
        while o < E:
            B = min(sizes[w % len(sizes)], E - o)
            got = srv.fold_take(src[o:], dst[o:], B, rec, cap, cnt)
            assert got <= B and int(cnt.item()) == srv.last_take_word, (w, B)
            rep.fold_records(rec, srv.last_take_word)  # rows | FAIL_BIT: the replay takes the verdict too
            rep.sync()
            o += B
            w += 1
        st = srv.window_server_stats()
        assert st["windows"] >= w // 2, st  # growth stops it; most windows still go through the server
        if kind == "cc":
            ov, olab = oracle_mod.cc_labels(hs, hd)
            for s in (srv, rep):
                v, lab = s.labels()
                assert np.array_equal(v, ov) and np.array_equal(lab, olab)
            assert srv.num_vertices() == len(ov)
        else:
            tok = oracle_mod.bip_truth(hs, hd)[0]
            assert srv.ok() == rep.ok() == tok


@pytest.mark.parametrize("kind", ["cc", "signed"])
def test_window_server_late_workgroup(kind):
    """a workgroup that becomes resident late keeps block 0 waiting (up to 8 x the
    idle limit) for the window it handed out; when that window completes the host posts the
    next one at once and block 0 takes it. Every other block must still be polling then (their
    own limit is 10 x the idle limit), or the next window never completes. The test build of
    the library (lib_testhooks: -DGS_TEST_LATE_WORKGROUP=400; the product kernel has no such
    branch) starts the last workgroup of every server launch 400 us late against a 100-us
    idle limit (GS_TESTING_SERVER_IDLE_US): with the old 2 x limit the other blocks left after
    200 us and the second window of every session failed. Idle gaps between some windows
    restart the server (a new late workgroup each time). Every window's rows replay to the
    summary, and both equal the oracle. A child process loads the test build."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GS_LIB_VARIANT="testhooks")
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "late_workgroup_check.py"), kind], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and "late workgroup ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
