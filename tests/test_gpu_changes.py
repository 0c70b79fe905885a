"""GPU: per-window change emission (gs_set_change_tracking / gs_take_changes_device;
SURVEY.md 8(f) row 3). The reference's Merger emits the whole cumulative summary per
window (SummaryAggregation.java:107-119) and FlattenSet flattens it into (vertex,
component) rows for a keyed sink (ConnectedComponentsExample.java:143-156). Here,
window by window, the emitted rows must be EXACTLY the vertices that are new or
whose canonical label changed (oracle labels before/after the window), and a sink
applying them must hold the oracle's labels of the whole prefix."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _oracle_state(oracle_mod, s, d):
    v, lab = oracle_mod.cc_labels(s, d)
    return dict(zip(v.tolist(), lab.tolist()))


def _run_windows(gs, oracle_mod, s, d, bounds, hint, exact=True, kind="cc"):
    sink = {}
    before = {}
    with gs.Summary(kind, capacity_hint=hint) as x:
        x.set_change_tracking(True)
        for lo, hi in zip(bounds[:-1], bounds[1:]):
            x.fold(s[lo:hi], d[lo:hi])
            v, lab = x.take_changes()
            after = _oracle_state(oracle_mod, s[:hi], d[:hi])
            rows = dict(zip(v.tolist(), lab.tolist()))
            assert len(rows) == len(v), "a vertex emitted twice in one window"
            changed = {k: l for k, l in after.items() if before.get(k) != l}
            for k, l in rows.items():
                assert after[k] == l, "wrong label emitted"
            assert set(changed) <= set(rows), "a changed vertex was not emitted"
            if exact:
                assert set(rows) == set(changed), "unchanged vertices emitted"
            sink.update(rows)
            assert sink == after
            before = after
    return sink


def test_changes_cc_default_stream_windows(gs, oracle_mod):
    # ConnectedComponentsExample default stream, 1000 ms windows (config 1): the sink
    # built from the emissions equals the derived golden after every window
    with open(os.path.join(GOLD, "derived.json")) as f:
        em = json.load(f)["cc_default_stream"]["emissions"]
    k = np.arange(1, 101, dtype=np.int64)
    win = (k * 100) // 1000
    bounds = [0] + [int(np.searchsorted(win, w, side="right")) for w in sorted(set(win.tolist()))]
    sink = {}
    with gs.Summary("cc", capacity_hint=256) as x:
        x.set_change_tracking(True)
        for wi, (lo, hi) in enumerate(zip(bounds[:-1], bounds[1:])):
            x.fold(k[lo:hi], k[lo:hi] + 2)
            v, lab = x.take_changes()
            sink.update(zip(v.tolist(), lab.tolist()))
            vs = np.array(sorted(sink), np.int64)
            assert oracle_mod.canonical_cc_string(vs, np.array([sink[q] for q in vs.tolist()], np.int64)) == em[wi]
    _run_windows(gs, oracle_mod, k, k + 2, bounds, 256)


@pytest.mark.parametrize("window", [1 << 10, 1 << 13])
def test_changes_rmat16_windows(gs, oracle_mod, window):
    s, d = oracle_mod.rmat_edges(0x5EED0016, 14, 0, 1 << 16, True)
    bounds = list(range(0, len(s), window)) + [len(s)]
    _run_windows(gs, oracle_mod, s, d, bounds, 1 << 16)  # no table rebuild: exact emissions


def test_changes_scan_path_for_large_relabels(gs, oracle_mod, knobs):
    # walk limit 8: every hooked component with more members is emitted by the scan
    # (a superset with unchanged members of the absorbing component); the sink state
    # must still equal the oracle after every window
    knobs(changes_walk_max=8)
    s, d = oracle_mod.rmat_edges(0x5EED0017, 12, 0, 1 << 14, True)
    bounds = list(range(0, len(s), 1 << 11)) + [len(s)]
    _run_windows(gs, oracle_mod, s, d, bounds, 1 << 12, exact=False)


def test_changes_through_table_growth_and_reset(gs, oracle_mod):
    # a tiny hint: the table is rebuilt during the stream (the next take emits every
    # vertex: a superset), then reset and reused (a pooled window summary)
    s, d = oracle_mod.er_edges(0x5EED00E5, 14, 0, 1 << 15, True)
    bounds = list(range(0, len(s), 1 << 12)) + [len(s)]
    _run_windows(gs, oracle_mod, s, d, bounds, 16, exact=False)
    with gs.Summary("cc", capacity_hint=1 << 14) as x:
        x.set_change_tracking(True)
        x.fold(s, d)
        x.take_changes()
        x.reset()
        x.fold(s[:100], d[:100])
        v, lab = x.take_changes()
        ov, olab = oracle_mod.cc_labels(s[:100], d[:100])
        o = np.argsort(v)
        assert np.array_equal(v[o], ov) and np.array_equal(lab[o], olab)


def test_changes_enabled_mid_stream(gs, oracle_mod):
    s, d = oracle_mod.rmat_edges(5, 12, 0, 1 << 13, True)
    with gs.Summary("cc", capacity_hint=1 << 12) as x:
        x.fold(s[:4000], d[:4000])
        x.set_change_tracking(True)  # existing vertices: the first take emits them all
        v, lab = x.take_changes()
        ov, olab = oracle_mod.cc_labels(s[:4000], d[:4000])
        o = np.argsort(v)
        assert np.array_equal(v[o], ov) and np.array_equal(lab[o], olab)
        sink = dict(zip(v.tolist(), lab.tolist()))
        x.fold(s[4000:], d[4000:])
        v, lab = x.take_changes()
        sink.update(zip(v.tolist(), lab.tolist()))
        assert sink == _oracle_state(oracle_mod, s, d)


def test_changes_host_arrays_equal_device_take(gs, oracle_mod):
    """gs_take_changes (host arrays, the JVM sink's entry point) emits exactly the rows
    gs_take_changes_device does, window by window, on two identical summaries; parity
    rows for the signed kind too."""
    s, d = oracle_mod.rmat_edges(0x5EED0018, 13, 0, 1 << 15, True)
    for kind in ("cc", "signed"):
        with gs.Summary(kind, capacity_hint=1 << 14) as a, gs.Summary(kind, capacity_hint=1 << 14) as b:
            a.set_change_tracking(True)
            b.set_change_tracking(True)
            for lo in range(0, len(s), 1 << 12):
                a.fold(s[lo:lo + (1 << 12)], d[lo:lo + (1 << 12)])
                b.fold(s[lo:lo + (1 << 12)], d[lo:lo + (1 << 12)])
                va, la = a.take_changes()
                vb, lb = b.take_changes_host()
                ia, ib = np.argsort(va), np.argsort(vb)
                assert np.array_equal(va[ia], vb[ib]) and np.array_equal(la[ia], lb[ib])
