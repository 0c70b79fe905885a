"""Young-table batches serialised vs pipelined (configs 2 and 4, one GPU).

A step = reset + 16 x 2^20-edge folds (+ the label pass / verdict read, as bench.py). Variant K
folds the first K batches of the empty table at pipelining depth 1, then the rest at depth 3
(K = 0: bench.py's step). The switch joins the lanes (one cross-queue wait). Prints ms per step
over alternating rounds."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402

E, B = 1 << 24, 1 << 20


def workload(name, dev):
    # the summary and its lanes first (bench.py: lanes created after torch's streams share a
    # hardware queue with them)
    s = gs.Summary("cc", capacity_hint=1 << 19) if name == "r20" else gs.Summary("signed", capacity_hint=1 << 20)
    s.set_pipelining(3)
    src = torch.empty(E, dtype=torch.int64, device=dev)
    dst = torch.empty(E, dtype=torch.int64, device=dev)
    if name == "r20":
        gs.gen_rmat(src, dst, 0, E, 20, 0x5EED0020, True)
        torch.cuda.synchronize(dev)
        return s, src, dst
    gs.gen_bip(src, dst, 0, E, 19, 0x5EED0B1B, [])
    torch.cuda.synchronize(dev)
    gs.relabel_first_appearance(src, dst, 2 << 19)
    torch.cuda.synchronize(dev)
    return s, src, dst


def main():
    dev = torch.device("cuda", 0)
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    for name in sys.argv[1:2]:  # one workload per process (r20 | bip)
        s, src, dst = workload(name, dev)
        vcap = (1 << 21) + 16
        out_v = torch.empty(vcap, dtype=torch.int64, device=dev)
        out_l = torch.empty(vcap, dtype=torch.int64, device=dev)

        def step(k):
            if k:
                s.set_pipelining(1)
            s.reset()
            for b in range(E // B):
                if k and b == k:
                    s.set_pipelining(3)
                s.fold_device(src[b * B:], dst[b * B:], n=B)
            if name == "r20":
                s.export_labels_device(out_v, out_l)
            else:
                s.ok()

        res = {}
        for rnd in range(3):
            for k in (0, 1, 2, 3):
                for _ in range(2):
                    step(k)
                s.sync()
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                for _ in range(steps):
                    step(k)
                s.sync()
                torch.cuda.synchronize(dev)
                res.setdefault(k, []).append((time.perf_counter() - t0) / steps * 1e3)
        for k, v in res.items():
            print("%s young-serial K=%d: ms/step %s" % (name, k, " ".join("%.3f" % x for x in v)), flush=True)
        s.close()


if __name__ == "__main__":
    main()
