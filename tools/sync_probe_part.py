"""Summary.sync() after the pipelined own folds of a partitioned group's rank, in the replay's
setting (N rank threads, collectives emulated, serialized token): times to Summary.sync(), to a
kernel-based wait (num_vertices) and to a device-wide synchronisation, with the group's phase
timing off and on."""
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

B = 1 << 20


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    per = 1 << 26
    E = per * N
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    for o in range(0, E, 1 << 26):
        gs.gen_rmat(src[o:], dst[o:], o, 1 << 26, 26, 0x5EED0026, True)
    torch.cuda.synchronize()
    gs.use_comm_emulation(True)
    F = gs.fake_comm()
    F.gs_fake_comm_set_serialize(1)
    uid = gs.group_unique_id()
    out = []

    def rank(r):
        F.gs_fake_comm_token(1)
        try:
            s = gs.Summary("cc", capacity_hint=1 << 25)
            s.set_pipelining(3)
            g = gs.PartGroup(s, uid, N, r, 1 << 25, 0)
            for rep, phases in enumerate((False, False, True, True)):
                g.reset()
                s.sync()
                g.set_phase_timing(phases)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for o in range(r * per, (r + 1) * per, B):
                    g.fold_device(src[o:], dst[o:], B)
                s.sync()
                a = time.perf_counter() - t0
                s.num_vertices()
                b = time.perf_counter() - t0
                torch.cuda.synchronize()
                c = time.perf_counter() - t0
                out.append((r, rep, phases, a * 1e3, b * 1e3, c * 1e3))
                g.combine()
            g.close()
            s.close()
        finally:
            F.gs_fake_comm_token(0)

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(N)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    F.gs_fake_comm_set_serialize(0)
    gs.use_comm_emulation(False)
    for r, rep, ph, a, b, c in sorted(out):
        print("rank %d pass %d phases %d: sync %.2f  num_vertices %.2f  device %.2f ms" % (r, rep, ph, a, b, c),
              flush=True)


if __name__ == "__main__":
    main()
