"""GPU: the BASELINE configs at their full sizes, checked against the oracle where the
oracle finishes in seconds and through size-independent properties everywhere else.

Config 3 (RMAT-26, 2^30 edges, 2^20-edge micro-batches, the bench's pipelined fold):
  * every edge's two endpoints carry the same label (batched find on the device);
  * every label is <= its vertex and is a fixed point (label(label) == label);
  * the vertex count equals the number of distinct endpoints;
  * the first 2^24 edges folded the same way equal the oracle bit for bit.
Config 5 (ER G(2^22, 2^26), 2^16-edge windows, delta records taken per window):
  * the per-window delta records, replayed into a second summary, reproduce the first
    summary exactly (the multi-GPU combine contract), checked at window 1, 8, 64 and
    at the end;
  * the first 64 windows equal the oracle at windows 1, 8 and 64;
  * the full stream passes the same properties as config 3.
Reference: DisjointSet.union/find (S/summaries/DisjointSet.java:66-118),
ConnectedComponentsTest.java:41 (canonical components)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _labels_of(summ, keys, chunk=1 << 26):
    import torch
    out = torch.empty_like(keys)
    found = torch.empty(keys.numel(), dtype=torch.uint8, device=keys.device)
    for o in range(0, keys.numel(), chunk):
        n = min(chunk, keys.numel() - o)
        summ.find_labels_device(keys[o:o + n], out[o:o + n], found[o:o + n], n=n)
    summ.sync()
    return out, found


def _check_properties(summ, src, dst):
    """Size-independent checks of a folded stream (all on the device)."""
    import torch
    nv = summ.num_vertices()
    chunk = 1 << 26
    for o in range(0, src.numel(), chunk):  # endpoints of every edge share a label
        n = min(chunk, src.numel() - o)
        ls, fs = _labels_of(summ, src[o:o + n])
        ld, fd = _labels_of(summ, dst[o:o + n])
        assert bool(fs.all()) and bool(fd.all()), "an endpoint is missing from the summary"
        assert bool(torch.equal(ls, ld)), "an edge joins two components"
        del ls, ld, fs, fd
    v = torch.empty(nv + 1, dtype=torch.int64, device=src.device)
    lab = torch.empty(nv + 1, dtype=torch.int64, device=src.device)
    got = summ.export_labels_device(v, lab)
    assert got == nv
    v, lab = v[:got], lab[:got]
    assert bool((lab <= v).all()), "a label above its vertex (labels are component minima)"
    ll, _ = _labels_of(summ, lab)
    assert bool(torch.equal(ll, lab)), "a label is not its own label"
    distinct = 0
    for lo_bits in range(4):  # distinct endpoints, in four slices of the id space (memory)
        parts = []
        for x in (src, dst):
            for o in range(0, x.numel(), chunk):
                y = x[o:o + chunk]
                parts.append(y[(y & 3) == lo_bits])
        distinct += int(torch.unique(torch.cat(parts)).numel())
        del parts
    assert distinct == nv, (distinct, nv)
    return nv


def test_config3_rmat26_full_stream(gs, oracle_mod):
    import torch
    scale, E, B = 26, 1 << 30, 1 << 20
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, scale, 0x5EED0026, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << (scale - 1)) as s:
        s.set_pipelining(3)  # as bench.py at one GPU
        for o in range(0, E, B):
            s.fold_device(src[o:], dst[o:], n=B)
        nv = _check_properties(s, src, dst)
        assert nv == 32802821  # the bench's vertices_labelled for this stream (BENCH_r01.json)
    m = 1 << 24  # the prefix the bench's CPU leg folds: bit-exact against the oracle
    with gs.Summary("cc", capacity_hint=1 << (scale - 1)) as s:
        s.set_pipelining(3)
        for o in range(0, m, B):
            s.fold_device(src[o:], dst[o:], n=B)
        v, lab = s.labels()
    hs, hd = src[:m].cpu().numpy(), dst[:m].cpu().numpy()
    ov, olab = oracle_mod.cc_labels(hs, hd)
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)


def test_config5_er_windows_with_delta_records(gs, oracle_mod):
    import torch
    logn, E, B = 22, 1 << 26, 1 << 16
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_er(src, dst, 0, E, logn, 0x5EED00E5, True)
    torch.cuda.synchronize()
    rec = torch.empty((B, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()  # filled on torch's stream; the library writes on the summary's
    checkpoints = {1, 8, 64, E // B}
    with gs.Summary("cc", capacity_hint=1 << logn) as s, gs.Summary("cc", capacity_hint=1 << logn) as rep:
        s.set_delta_tracking(True)
        for w in range(E // B):
            o = w * B
            s.fold_device(src[o:], dst[o:], n=B)
            s.take_delta_records(rec, B, cnt)
            s.sync()
            k = int(cnt.item())
            assert k <= B  # at most one record per folded edge
            rep.fold_records(rec, k)  # the records alone rebuild the summary
            rep.sync()  # rec is reused by the next take
            if w + 1 in checkpoints:
                v1, l1 = s.labels()
                v2, l2 = rep.labels()
                assert np.array_equal(v1, v2) and np.array_equal(l1, l2), "replay differs at window %d" % (w + 1)
                if w + 1 <= 64:
                    hs, hd = src[:o + B].cpu().numpy(), dst[:o + B].cpu().numpy()
                    ov, olab = oracle_mod.cc_labels(hs, hd)
                    assert np.array_equal(v1, ov) and np.array_equal(l1, olab), "oracle differs at window %d" % (w + 1)
        _check_properties(s, src, dst)


def _bip_first_appearance(gs, E, logside, inject):
    """Config 4's stream as SURVEY.md 8(d) specifies it: ids in first-appearance order."""
    import torch
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_bip(src, dst, 0, E, logside, 0x5EED0B1B, inject)
    torch.cuda.synchronize()
    gs.relabel_first_appearance(src, dst, 2 << logside)
    torch.cuda.synchronize()
    return src, dst


def test_config4_bipartite_full_stream(gs, oracle_mod):
    """Config 4 at full size: sides of 2^19, E = 2^24 in 2^20-edge windows, ids in
    first-appearance order. Odd-cycle variant (same-side edges injected at E/8, E/4, E/2,
    3E/4): the verdict flips in exactly the window of the first conflicting edge (truth:
    the oracle's parity union-find). Clean variant: bipartite, colouring equal to the
    truth."""
    import torch
    logside, E, B = 19, 1 << 24, 1 << 20
    inject = [E // 8, E // 4, E // 2, 3 * E // 4]
    src, dst = _bip_first_appearance(gs, E, logside, inject)
    first = oracle_mod.bip_first_failure(src.cpu().numpy(), dst.cpu().numpy())
    assert first >= 0
    with gs.Summary("signed", capacity_hint=1 << 20) as c:
        for o in range(0, E, B):
            c.fold_device(src[o:], dst[o:], n=B)
            assert c.ok() == (first >= o + B), (o, first)
    src, dst = _bip_first_appearance(gs, E, logside, [])
    with gs.Summary("signed", capacity_hint=1 << 20) as c:
        c.set_pipelining(3)
        for o in range(0, E, B):
            c.fold_device(src[o:], dst[o:], n=B)
        ok, comp, v, sign = c.colouring()
    tok, tcomp, tv, tsign = oracle_mod.bip_truth(src.cpu().numpy(), dst.cpu().numpy())
    assert ok and tok
    assert np.array_equal(comp, tcomp) and np.array_equal(v, tv) and np.array_equal(sign, tsign)


@pytest.mark.parametrize("variant", ["odd_cycle", "clean"])
def test_config4_prefix_equals_reference_candidates(gs, oracle_mod, variant):
    """on the first 2^15 edges of config 4's stream (first-appearance
    ids, one window, p = 1 -- the reference's exact regime) the GPU's
    output string equals the REFERENCE's: the quirk-exact restatement of
    Candidates.merge (Candidates.java:77-192, BipartitenessCheck.java:54-61), whose result
    must not diverge from the truth there."""
    logside, E, m = 19, 1 << 24, 1 << 15
    inject = [E // 8, E // 4, E // 2, 3 * E // 4] if variant == "odd_cycle" else []
    src, dst = _bip_first_appearance(gs, E, logside, inject)
    ps, pd = src[:m].cpu().numpy(), dst[:m].cpu().numpy()
    div = oracle_mod.bip_quirk_divergence(ps, pd)
    assert not div["diverges"]
    with gs.Summary("signed", capacity_hint=m) as c:
        c.fold_device(src[:m], dst[:m], n=m)
        got = oracle_mod.canonical_candidates_string(*c.colouring())
    assert got == div["quirk"]
