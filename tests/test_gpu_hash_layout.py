"""GPU: the slot table's line-grouped home slots (csrc/gs_device.hpp hash_slot: ids that
differ only in their low three bits share a 128-B line) under id families that stress that
layout -- dense ranges (whole lines full), groups of eight consecutive ids at random bases,
multiples of 8 (every id at offset 0 of its line), a stride of 2^20, and ids at the int64
extremes (INT64_MIN lives in the reserved slot). Each family is folded from a small capacity
hint, so the table grows and rehashes several times, and the labels must equal an
independent scipy restatement of DisjointSet's canonical labelling (the minimum id of each
component, S/summaries/DisjointSet.java:92-118); a signed summary's colouring of a
bipartite stream over the same ids must equal the two-colouring's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

I64 = np.iinfo(np.int64)


def _families():
    rng = np.random.default_rng(0x11E5)
    n = 1 << 14
    bases = np.unique(rng.integers(-(1 << 38), 1 << 38, n // 8, dtype=np.int64)) << 12  # (distinct; 2^12 apart)
    extremes = np.array([I64.min, I64.min + 1, I64.min + 7, I64.min + 8, -1, 0, 1, 7, 8,
                         I64.max - 8, I64.max - 7, I64.max - 1, I64.max], dtype=np.int64)
    return {
        "dense": np.arange(n, dtype=np.int64),
        "groups_of_8": (bases[:, None] + np.arange(8, dtype=np.int64)[None, :]).ravel(),
        "multiples_of_8": np.arange(n, dtype=np.int64) * 8,
        "stride_2^20": (np.arange(n, dtype=np.int64) - n // 2) << 20,
        "extremes": np.concatenate([extremes, rng.integers(I64.min, I64.max, n - len(extremes), dtype=np.int64)]),
    }


def _labels(u, v):
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components
    ids = np.unique(np.concatenate([u, v]))
    iu, iv = np.searchsorted(ids, u), np.searchsorted(ids, v)
    g = coo_matrix((np.ones(len(u)), (iu, iv)), shape=(len(ids), len(ids)))
    _, lab = connected_components(g, directed=False)
    mins = np.full(lab.max() + 1, I64.max)
    np.minimum.at(mins, lab, ids)
    return ids, mins[lab]


FAMILIES = ["dense", "groups_of_8", "multiples_of_8", "stride_2^20", "extremes"]


@pytest.mark.parametrize("family", FAMILIES)
def test_line_grouped_slots_cc_labels(gs, family):
    ids = _families()[family]
    rng = np.random.default_rng(len(family))
    m = 2 * len(ids)  # average degree 4: a giant component and many small ones
    u = rng.choice(ids, m)
    v = rng.choice(ids, m)
    with gs.Summary("cc", capacity_hint=1 << 8) as s:
        for k in range(0, m, 4096):
            s.fold(u[k:k + 4096], v[k:k + 4096])
        vv, lab = s.labels()
    ev, el = _labels(u, v)
    assert np.array_equal(vv, ev)
    assert np.array_equal(lab, el)


@pytest.mark.parametrize("family", ["dense", "groups_of_8", "extremes"])
def test_line_grouped_slots_signed_colouring(gs, family):
    ids = _families()[family]
    rng = np.random.default_rng(7 + len(family))
    side = rng.integers(0, 2, len(ids)).astype(bool)
    left, right = ids[side], ids[~side]
    m = 3 * len(ids)
    u = rng.choice(left, m)
    v = rng.choice(right, m)
    with gs.Summary("signed", capacity_hint=1 << 8) as s:
        s.fold(u, v)
        ok, comp, vv, sign = s.colouring()
    assert ok  # every edge crosses the two sides
    ev, el = _labels(u, v)
    o = np.lexsort((ev, el))
    assert np.array_equal(comp, el[o]) and np.array_equal(vv, ev[o])
    colour = dict(zip(ids.tolist(), side.tolist()))
    want = np.array([colour[int(x)] == colour[int(c)] for x, c in zip(ev[o], el[o])], dtype=sign.dtype)
    assert np.array_equal(sign, want)
