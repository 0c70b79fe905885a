"""Does Summary.sync() wait for pipelined folds when several host threads drive summaries?
Each of T threads owns a summary (pipelining 3) and, one thread at a time (a lock), folds 128 x
2^20 RMAT-26 edges and calls Summary.sync(); then a kernel-based wait (num_vertices) and a
device-wide synchronisation. Prints the three times per thread and pass."""
import os
import sys
import threading
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

E, B = 1 << 27, 1 << 20


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, E, 26, 0x5EED0026, True)
    torch.cuda.synchronize()
    lock = threading.Lock()
    out = []

    def run(t):
        with gs.Summary("cc", capacity_hint=1 << 25) as s:
            s.set_pipelining(3)
            for rep in range(3):
                with lock:
                    s.reset()
                    s.sync()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for o in range(0, E, B):
                        s.fold_device(src[o:], dst[o:], n=B)
                    s.sync()
                    a = time.perf_counter() - t0
                    s.num_vertices()
                    b = time.perf_counter() - t0
                    torch.cuda.synchronize()
                    c = time.perf_counter() - t0
                    out.append((t, rep, a * 1e3, b * 1e3, c * 1e3))

    ts = [threading.Thread(target=run, args=(t,)) for t in range(T)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    for t, rep, a, b, c in out:
        print("thread %d pass %d: sync %.2f  num_vertices %.2f  device %.2f ms" % (t, rep, a, b, c), flush=True)


if __name__ == "__main__":
    main()
