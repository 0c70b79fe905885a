"""Randomised parity soak (diagnostic, GPU): random streams, batchings, capacity hints,
pipelining depths and host-API interleavings folded through the HIP library, each case
checked against the oracle (CC: oracle.cc_labels; signed: oracle.bip_truth, verdict and
canonical colouring). Prints one line per case and a final JSON summary; stops at the
first mismatch with the case's seed so it can be replayed.
    python tools/parity_soak.py [--seconds 240] [--seed 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402
import oracle  # noqa: E402  (checker only)

I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1


def stream(rng, seed):
    fam = rng.choice(["rmat", "er", "bip", "sparse"], p=[0.35, 0.2, 0.25, 0.2])
    n = int(2 ** rng.uniform(4, 20))
    if fam == "rmat":
        s, d = oracle.rmat_edges(seed, int(rng.integers(6, 17)), 0, n, bool(rng.integers(2)))
    elif fam == "er":
        s, d = oracle.er_edges(seed, int(rng.integers(4, 17)), 0, n, bool(rng.integers(2)))
    elif fam == "bip":
        inject = sorted(set(int(x) for x in rng.integers(0, n, int(rng.integers(0, 3)))))
        s, d = oracle.bip_edges(seed, int(rng.integers(3, 15)), 0, n, inject)
    else:  # arbitrary 64-bit ids: extremes, self-loops, repeats
        pool = rng.integers(I64_MIN, I64_MAX, max(2, n // int(rng.integers(1, 16))), dtype=np.int64, endpoint=True)
        pool[: min(len(pool), 2)] = [I64_MIN, I64_MAX][: min(len(pool), 2)]
        s = rng.choice(pool, n)
        d = rng.choice(pool, n)
        loops = rng.random(n) < rng.uniform(0, 0.3)
        d[loops] = s[loops]
    return fam, np.ascontiguousarray(s, np.int64), np.ascontiguousarray(d, np.int64)


def fold_all(rng, summ, s, d, ts, td):
    """Fold the stream in random chunks through a random mix of entry points."""
    o, n = 0, len(s)
    while o < n:
        k = int(min(n - o, max(1, 2 ** rng.uniform(0, 21))))
        how = rng.random()
        if how < 0.6:
            summ.fold_device(ts[o:], td[o:], n=k)
        elif how < 0.9:
            summ.fold(s[o:o + k], d[o:o + k])
        else:  # strided device view: every edge of the chunk through an interleaved buffer
            inter = torch.empty((k, 2), dtype=torch.int64, device="cuda")
            inter[:, 0] = ts[o:o + k]
            inter[:, 1] = td[o:o + k]
            torch.cuda.synchronize()  # the copies ran on torch's stream, the fold runs on the summary's
            summ.fold_device(inter[:, 0], inter[:, 1], n=k, stride=2)
            summ.sync()
        if rng.random() < 0.05:
            summ.num_vertices()  # a host read in the middle of the stream
        o += k


def check(kind, summ, s, d):
    if kind == "cc":
        ov, olab = oracle.cc_labels(s, d)
        v, lab = summ.labels()
        return np.array_equal(v, ov) and np.array_equal(lab, olab)
    tok, tcomp, tv, tsign = oracle.bip_truth(s, d)
    ok, comp, v, sign = summ.colouring()
    if ok != tok:
        return False
    return not ok or (np.array_equal(comp, tcomp) and np.array_equal(v, tv) and np.array_equal(sign, tsign))


def run_case(seed, diag=False, partials=True):
    """One random case; returns (key, edges, exact). With diag, the partials of a
    combine / serialize case are checked on their own first and differences printed."""
    rng = np.random.default_rng(seed)
    fam, s, d = stream(rng, seed)
    kind = "signed" if (fam == "bip" or rng.random() < 0.2) else "cc"
    hint = int(2 ** rng.uniform(0, 21))
    depth = int(rng.integers(1, 5))
    ts, td = torch.from_numpy(s).cuda(), torch.from_numpy(d).cuda()
    mode = rng.choice(["plain", "reset", "combine", "serialize", "take"])
    key = "%s/%s/%s n=%d hint=%d depth=%d" % (kind, fam, mode, len(s), hint, depth)
    cut = None
    with gs.Summary(kind, capacity_hint=hint) as summ:
        if depth > 1:
            summ.set_pipelining(depth)
        if mode == "reset":  # a stale pass, reset, then the real one
            fold_all(rng, summ, d[: len(d) // 2], s[: len(s) // 2], td, ts)
            summ.reset()
            fold_all(rng, summ, s, d, ts, td)
        elif mode == "combine":  # two partials of a random split, combined (CombineCC / Candidates.merge)
            cut = int(rng.integers(0, len(s) + 1))
            with gs.Summary(kind, capacity_hint=hint) as other:
                fold_all(rng, summ, s[:cut], d[:cut], ts, td)
                fold_all(rng, other, s[cut:], d[cut:], ts[cut:], td[cut:])
                if diag and partials:
                    print("cut", cut, "partial A exact", check(kind, summ, s[:cut], d[:cut]),
                          "partial B exact", check(kind, other, s[cut:], d[cut:]),
                          "vertices", summ.num_vertices(), other.num_vertices(), flush=True)
                summ.combine(other)
        elif mode == "serialize":  # checkpoint half way, restore into a fresh summary, finish there
            cut = int(rng.integers(0, len(s) + 1))
            fold_all(rng, summ, s[:cut], d[:cut], ts, td)
            blob = summ.serialize()
            with gs.Summary(kind, capacity_hint=1) as restored:
                restored.deserialize(blob)
                if diag:
                    print("cut", cut, "restored exact", check(kind, restored, s[:cut], d[:cut]), flush=True)
                fold_all(rng, restored, s[cut:], d[cut:], ts[cut:], td[cut:])
                return key, len(s), check(kind, restored, s, d)
        elif mode == "take":  # latency-path windows (fold + take in one launch), replayed elsewhere
            summ.set_delta_tracking(True)
            w = max(int(2 ** rng.uniform(0, 16)), len(s) >> 12)  # at most 4096 windows per case
            cap = w + 16  # at most one record per folded edge
            rec = torch.empty((cap, 3), dtype=torch.int64, device="cuda")
            cnt = torch.empty(1, dtype=torch.int64, device="cuda")
            with gs.Summary(kind, capacity_hint=hint) as rep:
                for o in range(0, len(s), w):
                    got = summ.fold_take(ts[o:], td[o:], min(w, len(s) - o), rec, cap, cnt)
                    if got > cap:
                        return key, len(s), False
                    rep.fold_records(rec, summ.last_take_word)  # rows | FAIL_BIT: the verdict travels
                    rep.sync()  # rec is reused by the next take
                if not check(kind, rep, s, d):  # labels, or verdict + colouring, every case
                    return key, len(s), False
        else:
            fold_all(rng, summ, s, d, ts, td)
        good = check(kind, summ, s, d)
        if diag and not good and kind == "cc":
            ov, olab = oracle.cc_labels(s, d)
            v, lab = summ.labels()
            print("vertices gpu %d oracle %d" % (len(v), len(ov)), flush=True)
            if len(v) == len(ov):
                bad = np.nonzero((v != ov) | (lab != olab))[0]
                print("differing rows", len(bad), [(int(v[i]), int(lab[i]), int(ov[i]), int(olab[i])) for i in bad[:10]])
            else:
                extra = np.setdiff1d(v, ov)
                missing = np.setdiff1d(ov, v)
                print("extra", len(extra), extra[:5].tolist(), "missing", len(missing), missing[:5].tolist())
                if cut is not None:
                    a = np.union1d(s[:cut], d[:cut])
                    b = np.union1d(s[cut:], d[cut:])
                    print("cut", cut, "vertices A %d B %d; missing in A %d, in B %d, in both %d" % (
                        len(a), len(b), np.isin(missing, a).sum(), np.isin(missing, b).sum(),
                        (np.isin(missing, a) & np.isin(missing, b)).sum()), flush=True)
        return key, len(s), good


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--replay", type=int, default=None, help="run only this case seed, with diagnostics")
    ap.add_argument("--no-partials", action="store_true", help="replay: no host reads before the combine")
    a = ap.parse_args()
    if a.replay is not None:
        key, n, good = run_case(a.replay, diag=True, partials=not a.no_partials)
        print("replay", a.replay, key, "ok" if good else "MISMATCH", flush=True)
        sys.exit(0 if good else 1)
    t_end = time.time() + a.seconds
    cases, edges, by = 0, 0, {}
    while time.time() < t_end:
        seed = a.seed * 1000003 + cases
        key, n, good = run_case(seed)
        cases += 1
        edges += n
        k = key.split(" ")[0]
        by[k] = by.get(k, 0) + 1
        print("case %d seed %d %s %s" % (cases, seed, key, "ok" if good else "MISMATCH"), flush=True)
        if not good:
            print(json.dumps({"cases": cases, "edges": edges, "mismatch_seed": seed}))
            sys.exit(1)
    print(json.dumps({"cases": cases, "edges": edges, "all_exact": True, "by_kind_family_mode": by}))


if __name__ == "__main__":
    main()
