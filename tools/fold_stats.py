"""Per-micro-batch anatomy of a fold pass (diagnostic; VERDICT r4 item 2: the young-table phases).

Folds the stream of one BASELINE config batch after batch on ONE stream (no pipelining),
with HIP events around every k_fold launch, and prints per batch:
  fold_us, new vertices, and -- with the debug-counter build (GS_LIB_VARIANT=debug, made by
  `make -C gelly-streaming_amd debug`) -- key CASes issued / lost, agent-scope re-reads,
  shortcut edges, same-root edges, find loads, successful hooks, hook calls / iterations /
  failed hook CASes and extra linear probes.
The debug build's counters are same-address atomics: its times are not the product's. Run
the product build for times and the debug build for counts.

    python tools/fold_stats.py r20|bip|rmat26 [--batches N]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gsamd as gs  # noqa: E402


def stream(cfg, nb):
    B = 1 << 20
    if cfg == "bip":
        E = 1 << 24
        fs = torch.empty(E, dtype=torch.int64, device="cuda")
        fd = torch.empty(E, dtype=torch.int64, device="cuda")
        gs.gen_bip(fs, fd, 0, E, 19, 0x5EED0B1B, [])
        torch.cuda.synchronize()
        gs.relabel_first_appearance(fs, fd, 2 << 19)
        torch.cuda.synchronize()
        return "signed", 1 << 20, fs, fd, min(nb, E // B)
    scale, seed = (20, 0x5EED0020) if cfg == "r20" else (26, 0x5EED0026)
    E = min(16 << scale, nb * B)
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, scale, seed, True)
    torch.cuda.synchronize()
    return "cc", 1 << (scale - 1), src, dst, E // B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfg", choices=["r20", "bip", "rmat26"])
    ap.add_argument("--batches", type=int, default=16)
    ap.add_argument("--passes", type=int, default=2, help="the last pass is printed (the first sizes the table)")
    ap.add_argument("--hint-log2", type=int, default=0, help="capacity hint (log2 vertices; 0: the bench's)")
    a = ap.parse_args()
    kind, hint, src, dst, nb = stream(a.cfg, a.batches)
    if a.hint_log2:
        hint = 1 << a.hint_log2
    B = 1 << 20
    s = gs.Summary(kind, capacity_hint=hint)
    keys = None
    for p in range(a.passes):
        s.reset()
        s.sync()
        rows = []
        prev_c = s.debug_counters()
        prev_nv = 0
        for b in range(nb):
            s.set_profiling(True)
            n0, ms0 = s.kernel_stats("fold")
            s.fold_device(src[b * B:], dst[b * B:], n=B)
            s.sync()
            n1, ms1 = s.kernel_stats("fold")
            c = s.debug_counters()
            nv = s.num_vertices()
            d = {k: c[k] - prev_c[k] for k in c}
            base = s.counters()
            rows.append((b, (ms1 - ms0) * 1e3, nv - prev_nv, d, base))
            prev_c, prev_nv = c, nv
        s.set_profiling(False)
    keys = list(rows[0][3].keys())
    print("# %s: %d batches of 2^20 edges, table %d slots, vertices %d" % (a.cfg, nb, s.table_capacity(), prev_nv))
    print("batch fold_us new_v " + " ".join(keys) + " hook_calls hook_iters hook_cas_fail")
    prev_h = (0, 0, 0)
    for b, us, dv, d, base in rows:
        h = (base["hooks"], base["hook_iters"], base["cas_fail"])
        print("%5d %7.1f %7d " % (b, us, dv) + " ".join("%d" % d[k] for k in keys) + " %d %d %d" % tuple(
            h[i] - prev_h[i] for i in range(3)), flush=True)
        prev_h = h
    s.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
