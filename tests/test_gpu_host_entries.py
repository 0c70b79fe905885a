"""GPU: gs_fold_parity, the host entry GpuCandidates.merge uses for a general (not
one-edge) Candidates input: each vertex folded against its component's anchor with
parity = the two signs differ (S/summaries/Candidates.java:77-139). Colourings are
checked against an independent numpy/scipy restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _expect(u, v, colour):
    """canonical colouring: comp = min id of the component, sign = same colour as it"""
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    ids = np.unique(np.concatenate([u, v]))
    iu, iv = np.searchsorted(ids, u), np.searchsorted(ids, v)
    g = coo_matrix((np.ones(len(u)), (iu, iv)), shape=(len(ids), len(ids)))
    _, lab = connected_components(g, directed=False)
    mins = np.full(lab.max() + 1, np.iinfo(np.int64).max)
    np.minimum.at(mins, lab, ids)
    comp = mins[lab]
    cmap = dict(zip(ids.tolist(), [colour[int(x)] for x in ids]))
    sign = np.array([cmap[int(x)] == cmap[int(c)] for x, c in zip(ids, comp)], dtype=np.uint8)
    o = np.lexsort((ids, comp))
    return comp[o], ids[o], sign[o]


def test_fold_parity_components(gs):
    rng = np.random.default_rng(11)
    n = 1 << 12
    ids = rng.choice(np.arange(-(1 << 40), 1 << 40, 7919, dtype=np.int64), n, replace=False)
    colour = dict(zip(ids.tolist(), rng.integers(0, 2, n).tolist()))
    u = rng.choice(ids, 3 * n)
    v = rng.choice(ids, 3 * n)
    w = np.array([colour[int(a)] != colour[int(b)] for a, b in zip(u, v)], dtype=np.uint8)
    with gs.Summary("signed", capacity_hint=1 << 10) as s:
        s.fold_parity(u, v, w)
        ok, comp, vv, sign = s.colouring()
        assert ok
        ec, ev, es = _expect(u, v, colour)
        assert np.array_equal(comp, ec) and np.array_equal(vv, ev) and np.array_equal(sign, es)
        # one same-side pair inside a component whose colours differ: an odd cycle
        a = ev[0]
        b = next(int(x) for x, c in zip(ev, ec) if c == ec[0] and colour[int(x)] != colour[int(a)])
        s.fold_parity([a], [b], [0])
        assert not s.ok()
        assert s.colouring()[2].size == 0  # (false,{})
    with gs.Summary("cc", capacity_hint=1 << 10) as s:  # a CC summary ignores the parities
        s.fold_parity(u, v, w)
        vv, lab = s.labels()
        ec, ev, _ = _expect(u, v, colour)
        o = np.argsort(ev)
        assert np.array_equal(vv, ev[o]) and np.array_equal(lab, ec[o])


@pytest.mark.parametrize("pinned", [True, False])
def test_fold_host_pinned_and_pageable(gs, oracle_mod, pinned):
    """gs_fold from host memory: chunks of every size are copied by DMA straight from a
    pinned (hipHostMalloc'ed) caller buffer; pageable buffers take the staging path above
    2^18 edges. Both equal the oracle, and the caller may overwrite its buffer as soon as
    each call returns (the next call's data is written into the same buffer)."""
    import torch
    n, call = (3 << 20) + 12345, (1 << 20) + 777  # calls of more than one chunk, ragged tail
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, 20, 0x5EED0026, True)
    torch.cuda.synchronize()
    hs_all, hd_all = src.cpu().numpy(), dst.cpu().numpy()
    bs = torch.empty(call, dtype=torch.int64, pin_memory=pinned)
    bd = torch.empty(call, dtype=torch.int64, pin_memory=pinned)
    with gs.Summary("cc", capacity_hint=1 << 16) as s:  # small hint: growth mid-stream
        for o in range(0, n, call):
            m = min(call, n - o)
            bs[:m] = torch.from_numpy(hs_all[o:o + m])  # reuse of the caller's buffer
            bd[:m] = torch.from_numpy(hd_all[o:o + m])
            s.fold(bs.numpy()[:m], bd.numpy()[:m])
        v, lab = s.labels()
    ov, olab = oracle_mod.cc_labels(hs_all, hd_all)
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)
