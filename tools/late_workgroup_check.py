"""Child process of tests/test_gpu_window_take.py::test_window_server_late_workgroup: runs
against the test build of the library (GS_LIB_VARIANT=testhooks, whose window server
starts its last workgroup 400 us late). Prints "late workgroup ok" when every window's
rows replay to the summary and both equal the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gsamd as gs  # noqa: E402
import oracle as oracle_mod  # noqa: E402


def main(kind):
    assert os.environ.get("GS_LIB_VARIANT") == "testhooks", "run with GS_LIB_VARIANT=testhooks"
    gs.testing_set("server_idle_us", 100)
    import time
    import torch
    B, nw = 1 << 16, 12
    E = B * nw
    src = torch.empty(E, dtype=torch.int64, device="cuda")
    dst = torch.empty(E, dtype=torch.int64, device="cuda")
    if kind == "cc":
        gs.gen_er(src, dst, 0, E, 17, 0x5EED00E9, True)
    else:
        gs.gen_bip(src, dst, 0, E, 16, 0x5EED0B1F, [])
    torch.cuda.synchronize()
    hs, hd = src.cpu().numpy(), dst.cpu().numpy()
    rec = torch.empty((B + 16, 3), dtype=torch.int64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    with gs.Summary(kind, capacity_hint=1 << 18) as srv, gs.Summary(kind, capacity_hint=1 << 18) as rep:
        srv.set_delta_tracking(True)
        srv.set_window_server(True)
        for w in range(nw):
            srv.fold_take(src[w * B:], dst[w * B:], B, rec, B + 16, cnt)
            rep.fold_records(rec, srv.last_take_word)
            rep.sync()
            if w % 4 == 3:
                time.sleep(0.01)  # past every limit: the server leaves; the next window starts a new launch
        st = srv.window_server_stats()
        assert st["launches"] >= 3 and st["windows"] >= nw - 1, st
        if kind == "cc":
            ov, olab = oracle_mod.cc_labels(hs, hd)
            for s in (srv, rep):
                v, lab = s.labels()
                assert np.array_equal(v, ov) and np.array_equal(lab, olab)
        else:
            tok = oracle_mod.bip_truth(hs, hd)[0]
            assert srv.ok() == rep.ok() == tok
            a, b = srv.colouring(), rep.colouring()
            assert a[0] == b[0] and all(np.array_equal(x, y) for x, y in zip(a[1:], b[1:]))
            if tok:  # and the truth's colouring
                assert oracle_mod.canonical_candidates_string(*a) == oracle_mod.canonical_candidates_string(
                    *oracle_mod.bip_truth(hs, hd))
    print("late workgroup ok (%s)" % kind)


if __name__ == "__main__":
    main(sys.argv[1])
