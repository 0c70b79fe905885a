"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU restatement (gs_oracle.cpp).

The oracle is the parity checker for the HIP path and the CPU baseline for
bench.py. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import it; the product path (gelly-streaming_amd/) never does.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libgs_oracle.so")
_lib = None

_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_sz = ctypes.c_size_t


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.or_last_error.restype = ctypes.c_char_p
        L.or_rmat_edges.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, _i64p, _i64p]
        L.or_er_edges.argtypes = L.or_rmat_edges.argtypes
        L.or_bip_edges.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, _u64p, _sz, _i64p, _i64p]
        L.or_scramble_id.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_scramble_id.restype = ctypes.c_int64
        L.or_cc_labels.argtypes = [_i64p, _i64p, _sz, _i64p, _i64p, _sz]
        L.or_cc_labels.restype = _sz
        for f in (L.or_cc_dataflow, L.or_bip_dataflow):
            f.argtypes = [_i64p, _i64p, _i64p, _i32p, _sz, ctypes.c_int, ctypes.c_char_p, _sz, ctypes.POINTER(_sz)]
            f.restype = ctypes.c_int
        L.or_bip_truth.argtypes = [_i64p, _i64p, _sz, ctypes.POINTER(ctypes.c_int), _i64p, _i64p, _u8p, _sz]
        L.or_bip_truth.restype = _sz
        L.or_bip_first_failure.argtypes = [_i64p, _i64p, _sz]
        L.or_bip_first_failure.restype = ctypes.c_int64
        L.or_disjointset_unit_test.restype = ctypes.c_int
        L.or_cpu_baseline_cc.argtypes = [_i64p, _i64p, _sz, _sz]
        L.or_cpu_baseline_cc.restype = ctypes.c_double
        L.or_cpu_baseline_cc_threads.argtypes = [_i64p, _i64p, _sz, _sz, ctypes.c_int]
        L.or_cpu_baseline_cc_threads.restype = ctypes.c_double
        L.or_cpu_window_latency_cc.argtypes = [_i64p, _i64p, _sz, _sz,
                                               np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")]
        L.or_cpu_window_latency_cc.restype = None
        L.or_format_edges.argtypes = [_i64p, _i64p, _sz, ctypes.c_int, _u8p, _sz]
        L.or_format_edges.restype = _sz
        L.or_parse_edges.argtypes = [ctypes.c_char_p, _sz, ctypes.c_int, _i64p, _i64p, _sz,
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64)]
        L.or_cpu_baseline_bip.argtypes = [_i64p, _i64p, _sz]
        L.or_cpu_baseline_bip.restype = ctypes.c_double
        _lib = L
    return _lib


def _arr(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int64))


# ---------------- generators (independent CPU implementation of the stream spec) ----------------
def rmat_edges(seed, scale, start, count, scramble=True):
    s = np.empty(count, np.int64)
    d = np.empty(count, np.int64)
    lib().or_rmat_edges(seed, scale, start, count, 1 if scramble else 0, s, d)
    return s, d


def er_edges(seed, logn, start, count, scramble=True):
    s = np.empty(count, np.int64)
    d = np.empty(count, np.int64)
    lib().or_er_edges(seed, logn, start, count, 1 if scramble else 0, s, d)
    return s, d


def bip_edges(seed, logside, start, count, inject=()):
    s = np.empty(count, np.int64)
    d = np.empty(count, np.int64)
    inj = np.ascontiguousarray(np.sort(np.asarray(inject, dtype=np.uint64)))
    lib().or_bip_edges(seed, logside, start, count, inj, len(inj), s, d)
    return s, d


def scramble_id(raw, seed):
    return lib().or_scramble_id(raw, seed)


# ---------------- CC ----------------
def cc_labels(src, dst):
    """Canonical labels of the whole stream folded by the DisjointSet restatement.
    Returns (vertices sorted ascending, label = min id of the component)."""
    src, dst = _arr(src), _arr(dst)
    n = lib().or_cc_labels(src, dst, len(src), np.empty(0, np.int64), np.empty(0, np.int64), 0)
    v = np.empty(n, np.int64)
    lab = np.empty(n, np.int64)
    lib().or_cc_labels(src, dst, len(src), v, lab, n)
    return v, lab


def _dataflow(fn, src, dst, win, part, transient):
    src, dst = _arr(src), _arr(dst)
    win = _arr(win if win is not None else np.zeros(len(src)))
    part = np.ascontiguousarray(np.asarray(part if part is not None else np.zeros(len(src)), dtype=np.int32))
    ln = _sz(0)
    rc = fn(src, dst, win, part, len(src), 1 if transient else 0, None, 0, ctypes.byref(ln))
    if rc < 0:
        raise RuntimeError(lib().or_last_error().decode())
    buf = ctypes.create_string_buffer(ln.value + 1)
    rc = fn(src, dst, win, part, len(src), 1 if transient else 0, buf, ln.value + 1, ctypes.byref(ln))
    if rc != 0:
        raise RuntimeError(lib().or_last_error().decode())
    out = buf.value.decode()
    return out.split("\n") if out else []


def cc_dataflow(src, dst, win=None, part=None, transient=False):
    """SummaryBulkAggregation + ConnectedComponents emulation: one canonical
    DisjointSet string per window emission."""
    return _dataflow(lib().or_cc_dataflow, src, dst, win, part, transient)


def bip_dataflow(src, dst, win=None, part=None, transient=False):
    """SummaryBulkAggregation + BipartitenessCheck emulation over the quirk-exact
    Candidates restatement: Candidates.toString() per window emission."""
    return _dataflow(lib().or_bip_dataflow, src, dst, win, part, transient)


def bip_truth(src, dst):
    """Ground truth (parity union-find): (ok, comp[], v[], sign[]) sorted by (comp, v)."""
    src, dst = _arr(src), _arr(dst)
    ok = ctypes.c_int(0)
    cap = 2 * len(src) + 1
    comp = np.empty(cap, np.int64)
    v = np.empty(cap, np.int64)
    sign = np.empty(cap, np.uint8)
    n = lib().or_bip_truth(src, dst, len(src), ctypes.byref(ok), comp, v, sign, cap)
    return bool(ok.value), comp[:n], v[:n], sign[:n]


def bip_first_failure(src, dst):
    src, dst = _arr(src), _arr(dst)
    return int(lib().or_bip_first_failure(src, dst, len(src)))


def disjointset_unit_test():
    return lib().or_disjointset_unit_test()


# ---------------- CPU baseline ----------------
def cpu_baseline_cc(src, dst, window, threads=1):
    src, dst = _arr(src), _arr(dst)
    if threads <= 1:
        return lib().or_cpu_baseline_cc(src, dst, len(src), window)
    return lib().or_cpu_baseline_cc_threads(src, dst, len(src), window, threads)


def format_edges(src, dst, sep=0):
    """Edge-list text ("src<sep>dst\\n" per edge) as a numpy uint8 array (test/bench input)."""
    src, dst = _arr(src), _arr(dst)
    out = np.empty(42 * len(src) + 1, np.uint8)
    n = lib().or_format_edges(src, dst, len(src), sep, out, len(out))
    return out[:n]


def parse_edges(text, sep=0):
    """Reference source-map semantics (split + Long.parseLong per readTextFile line):
    (src, dst, n_lines, bad_line); bad_line = first malformed line or -1."""
    text = bytes(text)
    cap = text.count(b"\n") + 1
    src = np.zeros(cap, np.int64)
    dst = np.zeros(cap, np.int64)
    n = ctypes.c_uint64(0)
    bad = ctypes.c_int64(-1)
    lib().or_parse_edges(text, len(text), sep, src, dst, cap, ctypes.byref(n), ctypes.byref(bad))
    return src[:n.value], dst[:n.value], int(n.value), int(bad.value)


def cpu_window_latency_cc(src, dst, window):
    """Seconds per window (fold + CombineCC/Merger) of the 1-thread restatement."""
    src, dst = _arr(src), _arr(dst)
    out = np.zeros((len(src) + window - 1) // window, np.float64)
    lib().or_cpu_window_latency_cc(src, dst, len(src), window, out)
    return out


def cpu_baseline_bip(src, dst):
    src, dst = _arr(src), _arr(dst)
    return lib().or_cpu_baseline_bip(src, dst, len(src))


def bip_quirk_divergence(src, dst, win=None, part=None):
    """SURVEY.md 8(a) contract (ii): does the reference's Candidates (quirk-exact
    restatement, O(E x components)) diverge from the truth on this stream? Returns
    {"quirk": its final emission, "truth": the canonical truth string, "diverges"}.
    Candidates.merge's order / window bugs: Candidates.java:77-139,176."""
    q = bip_dataflow(src, dst, win, part)
    quirk = q[-1] if q else "(true,{})"
    truth = canonical_candidates_string(*bip_truth(src, dst))
    return {"quirk": quirk, "truth": truth, "diverges": quirk != truth}


def _mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def label_digest(v, lab, parity=None):
    """Restatement of gs_digest (include/gs_summary.h) over exported (v, label, parity)
    rows: sum mod 2^64 of mix64(v ^ C1) * mix64(label + parity * C2). Checker only."""
    v = np.asarray(v, dtype=np.int64).view(np.uint64)
    lab = np.asarray(lab, dtype=np.int64).view(np.uint64)
    p = np.zeros(len(v), np.uint64) if parity is None else np.asarray(parity).astype(np.uint64)
    with np.errstate(over="ignore"):
        a = _mix64(v ^ np.uint64(0x243F6A8885A308D3))
        b = _mix64(lab + np.where(p != 0, np.uint64(0x13198A2E03707344), np.uint64(0)))
        return int(np.sum(a * b, dtype=np.uint64))


# ---------------- canonical formatting shared by tests ----------------
def canonical_cc_string(v, lab):
    """'{min=[members ascending], ...}' -- DisjointSet.toString() shape."""
    comps = {}
    for a, b in zip(np.asarray(v).tolist(), np.asarray(lab).tolist()):
        comps.setdefault(b, []).append(a)
    parts = []
    for k in sorted(comps):
        parts.append("%d=[%s]" % (k, ", ".join(str(x) for x in sorted(comps[k]))))
    return "{" + ", ".join(parts) + "}"


def canonical_candidates_string(ok, comp, v, sign):
    """Candidates.toString() of the canonical colouring: '(ok,{c={v=(v,sign), ...}, ...})'."""
    if not ok:
        return "(false,{})"
    comps = {}
    for c, x, s in zip(np.asarray(comp).tolist(), np.asarray(v).tolist(), np.asarray(sign).tolist()):
        comps.setdefault(c, []).append((x, bool(s)))
    parts = []
    for c in sorted(comps):
        inner = ", ".join("%d=(%d,%s)" % (x, x, "true" if s else "false") for x, s in sorted(comps[c]))
        parts.append("%d={%s}" % (c, inner))
    return "(true,{" + ", ".join(parts) + "})"


def cc_test_parser(emissions):
    """ConnectedComponentsTest.parser (ConnectedComponentsTest.java:65-81): take the
    last emission, split on '=', keep the '[...]' lists, sort the lines."""
    r = emissions[-1]
    out = []
    for g in r.split("="):
        if "[" in g:
            k = g.split("]")
            out.append(k[0][1:])
    return sorted(out)
