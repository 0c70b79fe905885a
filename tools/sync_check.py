"""Does gs_sync wait for pipelined (tracked) folds of a partitioned group's local forest?
Times 128 x 2^20-edge folds of one rank (N = 1, collectives emulated) closed by Summary.sync()
against the same closed by a device-wide synchronisation, bulk and 2^22-edge windows."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402


def main():
    E, B = 1 << 27, 1 << 20
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, 26, 0x5EED0026, True)
    torch.cuda.synchronize()
    gs.use_comm_emulation(True)
    for W in (0, 1 << 22):
        with gs.Summary("cc", capacity_hint=1 << 25) as s:
            s.set_pipelining(3)
            g = gs.PartGroup(s, gs.group_unique_id(), 1, 0, 1 << 25, W)
            for how in ("summary.sync", "device", "summary.sync", "device"):
                g.reset()
                torch.cuda.synchronize()
                t_fold, t_all = 0.0, time.perf_counter()
                step = W or E
                for w0 in range(0, E, step):
                    t0 = time.perf_counter()
                    for o in range(w0, w0 + step, B):
                        g.fold_device(src[o:], dst[o:], B)
                    if how == "device":
                        torch.cuda.synchronize()
                    else:
                        s.sync()
                    t_fold += time.perf_counter() - t0
                    g.combine()
                torch.cuda.synchronize()
                print("window %8d  %-13s folds %7.2f ms  pass %7.2f ms" % (W, how, t_fold * 1e3,
                                                                            (time.perf_counter() - t_all) * 1e3),
                      flush=True)
            g.close()
    gs.use_comm_emulation(False)


if __name__ == "__main__":
    main()
