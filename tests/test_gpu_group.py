"""GPU: the native RCCL group (include/gs_group.h) at one rank: fold + stage +
ncclAllGather + header-driven capacity + backlog drain, on the summary's stream.
(Several ranks need several GPUs: RCCL refuses two ranks on one device; the
multi-rank protocol itself is covered by test_gpu_distributed.py / the gloo tests.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("first_cap", [0, 64])
def test_group_single_rank_matches_oracle(gs, oracle_mod, monkeypatch, first_cap):
    import torch
    monkeypatch.setenv("GS_GROUP_RETUNE", "2")
    n, B = 1 << 17, 1 << 12
    src = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int64, device="cuda")
    gs.gen_rmat(src, dst, 0, n, 15, 0x5EED0026, True)
    torch.cuda.synchronize()
    with gs.Summary("cc", capacity_hint=1 << 15) as s:
        g = gs.Group(s, gs.group_unique_id(), 1, 0, B, first_cap)
        for i in range(0, n, B):
            g.fold_device(src[i:], dst[i:], B)
        g.finish()
        st = g.stats()
        assert st["exchanges"] >= n // B
        v, lab = s.labels()
        g.close()
    ov, olab = oracle_mod.cc_labels(src.cpu().numpy(), dst.cpu().numpy())
    assert np.array_equal(v, ov) and np.array_equal(lab, olab)
