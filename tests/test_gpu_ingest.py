"""GPU parity of the text edge ingest (include/gs_ingest.h) against the oracle's
restatement of the reference's source map (split + Long.parseLong per line,
ConnectedComponentsExample.java:109-118, BipartitenessCheckExample.java:97-106)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

I64_MIN = -(1 << 63)
I64_MAX = (1 << 63) - 1


def _random_text(rng, nlines, sep):
    s = b"\t" if sep == 1 else b" "
    seps = [b" ", b"\t", b"\x0b", b"\x0c"] if sep == 0 else [b"\t"]
    good_vals = [0, 1, -1, 7, I64_MAX, I64_MIN, 123456789012345678]
    lines = []
    for i in range(nlines):
        r = rng.random()
        a = int(rng.choice(good_vals)) if rng.random() < 0.2 else int(rng.integers(-(10 ** 12), 10 ** 12))
        b = int(rng.integers(-(10 ** 18), 10 ** 18))
        sp = seps[int(rng.integers(len(seps)))]
        if r < 0.80:
            ln = b"%d%s%d" % (a, sp, b)
        elif r < 0.85:
            ln = b"+%d%s%d" % (abs(a), sp, b)
        elif r < 0.88:
            ln = b"%d%s%d%s%s" % (a, sp, b, s, b"x" * int(rng.integers(1, 700)))  # long ignored 3rd field
        elif r < 0.91:
            ln = b"%d%s%d\r" % (a, sp, b)
        elif r < 0.93:
            ln = b"%d%s%d%s" % (a, sp, b, sp)  # trailing separator
        else:  # malformed variants
            bad = [b"", b"%d" % a, s + b"%d%s%d" % (a, s, b), b"%d%s%s%d" % (a, s, s, b), b"%da%s%d" % (a, s, b),
                   b"9223372036854775808%s1" % s, b"-%s5" % s, b"1%s-9223372036854775809" % s]
            ln = bad[int(rng.integers(len(bad)))]
        lines.append(ln)
    text = b"\n".join(lines)
    if rng.random() < 0.5:
        text += b"\n"
    return text


def _gpu_parse(gs, text, sep, offset=0):
    import torch
    buf = torch.zeros(len(text) + offset, dtype=torch.uint8, device="cuda")
    if text:
        buf[offset:] = torch.frombuffer(bytearray(text), dtype=torch.uint8).cuda()
    view = buf[offset:]
    cap = text.count(b"\n") + 1
    src = torch.zeros(cap, dtype=torch.int64, device="cuda")
    dst = torch.zeros(cap, dtype=torch.int64, device="cuda")
    n, bad = gs.parse_edges_device(view, src, dst, sep)
    torch.cuda.synchronize()
    return src.cpu().numpy()[:n], dst.cpu().numpy()[:n], n, bad


@pytest.mark.parametrize("sep", [0, 1])
@pytest.mark.parametrize("seed,nlines,offset", [(1, 50, 0), (2, 20000, 0), (3, 150000, 0), (4, 30000, 1),
                                                (5, 30000, 7)])
def test_parse_matches_oracle(gs, oracle_mod, sep, seed, nlines, offset):
    rng = np.random.default_rng(seed)
    text = _random_text(rng, nlines, sep)
    es, ed, en, eb = oracle_mod.parse_edges(text, sep)
    s, d, n, b = _gpu_parse(gs, text, sep, offset)
    assert (n, b) == (en, eb)
    assert np.array_equal(s, es) and np.array_equal(d, ed)


@pytest.mark.parametrize("text", [b"", b"\n", b"1 2", b"1 2\n", b"1 2\n\n", b"\n1 2", b"1 2\r", b"1 2\r\n3 4\r\n",
                                  b"-9223372036854775808 9223372036854775807\n"])
def test_parse_edge_cases(gs, oracle_mod, text):
    for sep in (0, 1):
        es, ed, en, eb = oracle_mod.parse_edges(text, sep)
        s, d, n, b = _gpu_parse(gs, text, sep)
        assert (n, b) == (en, eb), (text, sep)
        assert np.array_equal(s, es) and np.array_equal(d, ed)


def test_fold_text_rmat_chunks_and_malformed(gs, oracle_mod):
    # > 16 MiB of text: several ingest chunks, each cut at a line boundary
    s, d = oracle_mod.rmat_edges(0x5EED0016, 16, 0, 1 << 20, True)
    text = b"\n".join(b"%d %d" % (a, b) for a, b in zip(s.tolist(), d.tolist())) + b"\n"
    assert len(text) > (16 << 20)
    with gs.Summary("cc", capacity_hint=1 << 16) as ds:
        assert ds.fold_text(text) == len(s)
        v, lab = ds.labels()
        ov, olab = oracle_mod.cc_labels(s, d)
        assert np.array_equal(v, ov) and np.array_equal(lab, olab)
    # a malformed line deep in the stream: GS_ERR_PARSE naming its line index
    lines = text.split(b"\n")
    k = 700001
    lines[k] = b"12 x"
    bad_text = b"\n".join(lines)
    with gs.Summary("cc", capacity_hint=1 << 16) as ds:
        with pytest.raises(gs.GSError) as e:
            ds.fold_text(bad_text)
        assert e.value.code == gs.GS_ERR_PARSE and str(k) in str(e.value)
    # tab-separated (BipartitenessCheckExample format) into a signed summary
    b0, b1 = oracle_mod.bip_edges(0x5EED0B1B, 12, 0, 1 << 14, [])
    tsv = b"\n".join(b"%d\t%d" % (a, b) for a, b in zip(b0.tolist(), b1.tolist()))
    with gs.Summary("signed", capacity_hint=1 << 13) as c, gs.Summary("signed", capacity_hint=1 << 13) as ref:
        assert c.fold_text(tsv, gs.SEP_TAB) == len(b0)
        ref.fold(b0, b1)
        ca, cb = c.colouring(), ref.colouring()
        assert ca[0] == cb[0] and all(np.array_equal(x, y) for x, y in zip(ca[1:], cb[1:]))


@pytest.mark.parametrize("sep", [0, 1])
def test_parse_window_boundaries_and_junk(gs, oracle_mod, sep):
    """Lines around the fast parser's 48-byte register window (padded with leading
    zeros and trailing fields to every length 1..80), signs, '\\r' placements and random
    byte junk, each against the oracle's split + Long.parseLong restatement."""
    rng = np.random.default_rng(11 + sep)
    s = b"\t" if sep == 1 else b" "
    lines = []
    for L in range(1, 81):
        for form in range(6):
            a = b"-9223372036854775808" if form == 0 else b"%d" % int(rng.integers(-(10 ** 9), 10 ** 9))
            b = b"9223372036854775807" if form == 1 else b"+%d" % int(rng.integers(0, 10 ** 12))
            core = a + s + b
            if form == 2:  # leading zeros up to the length
                ln = b"0" * max(0, L - len(core)) + core
            elif form == 3:  # ignored third field up to the length
                ln = core + s + b"z" * max(0, L - len(core) - 1)
            elif form == 4:  # '\r' before the end, or inside
                ln = core + b"\r" if L % 2 else a + b"\r" + b
            else:  # digits of field 1 up to the length (overflow past 19 digits)
                ln = a + s + b"1" * max(1, L - len(a) - 1)
            lines.append(ln)
    junk = b"0123456789 \t\r+-x"
    for _ in range(3000):
        n = int(rng.integers(0, 60))
        lines.append(bytes(junk[int(i)] for i in rng.integers(0, len(junk), n)))
    rng.shuffle(lines)
    for tail in (b"", b"\n"):
        text = b"\n".join(lines) + tail
        es, ed, en, eb = oracle_mod.parse_edges(text, sep)
        got = _gpu_parse(gs, text, sep)
        assert (got[2], got[3]) == (en, eb)
        assert np.array_equal(got[0], es) and np.array_equal(got[1], ed)
    # every line on its own (first-malformed index = 0 or none), incl. the text's end
    for ln in lines[:400]:
        es, ed, en, eb = oracle_mod.parse_edges(ln, sep)
        got = _gpu_parse(gs, ln, sep)
        assert (got[2], got[3]) == (en, eb), ln
        assert np.array_equal(got[0], es) and np.array_equal(got[1], ed), ln


def _text_with_newline_at(pos, end):
    """Lines "0..01 2" (zero-padded to 30-80 bytes) whose newlines include byte `pos`;
    the text is cut at `end` bytes (its last line may lack a newline)."""
    out, k = bytearray(), 0

    def line(n):  # n bytes before the newline
        out.extend(b"0" * (n - 3) + b"1 2\n")

    while pos - len(out) > 80:
        k += 1
        line(30 + (k * 7) % 21)
    line(pos - len(out))  # 30..80 bytes: its newline is byte pos
    while len(out) < end:
        k += 1
        line(30 + (k * 7) % 21)
    return bytes(out[:end])


@pytest.mark.parametrize("sep", [0, 1])
def test_parse_newlines_at_tile_edges(gs, oracle_mod, sep):
    """A newline at every byte around the parser's tile edges (8 and 16 KiB multiples,
    and the 512 bytes of the next tile it stages), and texts that end there with and
    without a last newline: line count, values and first malformed line vs the oracle."""
    for base in (8192, 16384, 16384 + 512, 32768, 49152):
        for d in range(-3, 4):
            pos = base + d
            for end in (pos, pos + 1, pos + 700):
                text = _text_with_newline_at(pos, end)
                if sep == 1:
                    text = text.replace(b" ", b"\t")
                assert end <= pos or text[pos] == 10
                es, ed, en, eb = oracle_mod.parse_edges(text, sep)
                got = _gpu_parse(gs, text, sep)
                assert (got[2], got[3]) == (en, eb), (base, d, end)
                assert np.array_equal(got[0], es) and np.array_equal(got[1], ed), (base, d, end)


def test_parse_malformed_then_clean_reuses_scratch(gs, oracle_mod):
    """The one-pass parse does not reset its malformed-line word per call: the previous
    parse's result kernel does. A parse that reports a malformed line, then clean texts
    of growing and shrinking sizes (fewer tiles than before: stale status words beyond
    the new tile count are never read), each report exactly the oracle's result."""
    rng = np.random.default_rng(11)
    texts = [_random_text(rng, 40000, 0) + b"12 x\n" + _random_text(rng, 100, 0), _random_text(rng, 40000, 0),
             _random_text(rng, 300, 0), b"1 2\nnot a line\n", _random_text(rng, 70000, 0), _random_text(rng, 5, 0)]
    for text in texts:
        es, ed, en, eb = oracle_mod.parse_edges(text, 0)
        s, d, n, b = _gpu_parse(gs, text, 0)
        assert (n, b) == (en, eb), (len(text), n, b, en, eb)
        assert np.array_equal(s, es) and np.array_equal(d, ed)


def test_parse_profiling_counts_kernel_time(gs):
    """gs_parse_set_profiling / gs_parse_profile (the bench's roofline timing): each
    parse adds its kernel time; turning it on again starts from zero."""
    rng = np.random.default_rng(12)
    text = _random_text(rng, 20000, 0)
    gs.parse_set_profiling(True)
    for _ in range(3):
        _gpu_parse(gs, text, 0)
    us, n = gs.parse_profile()
    assert n == 3 and us > 0.0
    gs.parse_set_profiling(True)
    assert gs.parse_profile() == (0.0, 0)
    gs.parse_set_profiling(False)
    _gpu_parse(gs, text, 0)
    assert gs.parse_profile()[1] == 0


def test_parse_release_frees_the_cache_and_parses_again(gs, oracle_mod):
    """gs_parse_release frees the thread's parse cache (device scratch, mapped record,
    timing events); the next parse rebuilds it and is still exact, a second release in a row is a
    no-op, and a worker thread that parses and releases leaves no allocation behind (the device's
    free memory returns to where it was)."""
    import threading
    import torch
    rng = np.random.default_rng(13)
    text = _random_text(rng, 30000, 0)
    es, ed, en, eb = oracle_mod.parse_edges(text, 0)
    for _ in range(2):
        s, d, n, b = _gpu_parse(gs, text, 0)
        assert (n, b) == (en, eb) and np.array_equal(s, es) and np.array_equal(d, ed)
        gs.parse_release()
        gs.parse_release()
    big = _random_text(rng, 400000, 0)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    err = []

    def worker():
        try:
            _gpu_parse(gs, big, 0)
            gs.parse_release()
        except Exception as e:  # noqa: BLE001 -- reported below
            err.append(e)

    t = threading.Thread(target=worker)
    t.start()
    t.join()
    assert not err, err
    torch.cuda.synchronize()
    # the worker's text and outputs are torch tensors (cached by torch's allocator, not returned);
    # the library's scratch of ~1.25 x the text went back to the device
    torch.cuda.empty_cache()
    assert torch.cuda.mem_get_info()[0] >= free0 - (1 << 20)


@pytest.mark.parametrize("offset", [0, 1, 7])
def test_parse_lookback_fallback_counts_directly(gs, oracle_mod, offset, knobs):
    """a tile whose predecessors have not published within the look-back's timeout
    counts the '\\n' before it itself (16-byte loads across the wave, an unaligned head and
    tail byte by byte). GS_TESTING_PARSE_LB_TIMEOUT_US = 0 makes every tile that finds an unpublished
    predecessor take that path; the result is still the oracle's, for aligned and unaligned
    texts of many tiles."""
    rng = np.random.default_rng(17 + offset)
    knobs(parse_lb_timeout_us=0)
    for nlines in (3000, 120000):
        text = _random_text(rng, nlines, 0)
        es, ed, en, eb = oracle_mod.parse_edges(text, 0)
        s, d, n, b = _gpu_parse(gs, text, 0, offset)
        assert (n, b) == (en, eb), (nlines, offset, n, b, en, eb)
        assert np.array_equal(s, es) and np.array_equal(d, ed)



def test_parse_sequence_reuses_cleared_status_words(gs, oracle_mod):
    """The one-pass parse leaves its tiles' status words zero for the next parse (k_parse_finish
    clears them with the result), so parses after the first run without a fill. A sequence of
    texts of different tile counts on one cached scratch -- large, small, large again, unaligned,
    malformed, empty, large -- must each equal the oracle: a status word left over from a longer
    parse would hand a later tile a wrong line number."""
    rng = np.random.default_rng(0x5EC)
    sizes = [(150000, 0), (2000, 0), (150000, 3), (40000, 1), (0, 0), (160000, 0), (700, 5)]
    for nlines, offset in sizes:
        text = _random_text(rng, nlines, 0) if nlines else b""
        es, ed, en, eb = oracle_mod.parse_edges(text, 0)
        s, d, n, b = _gpu_parse(gs, text, 0, offset)
        assert (n, b) == (en, eb), (nlines, offset, n, b, en, eb)
        assert np.array_equal(s, es) and np.array_equal(d, ed), (nlines, offset)
    # the host text path (gs_fold_text, the summary's own scratch), texts of different sizes
    for nlines in (60000, 900, 60000):
        a = rng.integers(-(10 ** 12), 10 ** 12, nlines)
        b = rng.integers(0, 5000, nlines)
        text = b"\n".join(b"%d %d" % (int(x), int(y)) for x, y in zip(a, b)) + b"\n"
        es, ed, en, eb = oracle_mod.parse_edges(text, 0)
        assert eb == -1 and en == nlines
        with gs.Summary("cc", capacity_hint=1 << 16) as summ:
            assert summ.fold_text(text) == nlines
            assert summ.num_vertices() == len(np.unique(np.concatenate([es, ed])))
