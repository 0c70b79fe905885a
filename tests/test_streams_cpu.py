"""CPU: stream preparation shared by bench.py and the GPU tests.

relabel_first_appearance renames a stream's ids to 1, 2, 3, ... in order of first
appearance (the reference's exact regime); it is
checked here against a plain dictionary restatement on torch CPU tensors."""
import numpy as np
import pytest


def _dict_relabel(s, d):
    ids = {}
    for a, b in zip(s.tolist(), d.tolist()):
        for x in (a, b):
            ids.setdefault(x, len(ids) + 1)
    return np.array([ids[x] for x in s.tolist()]), np.array([ids[x] for x in d.tolist()])


@pytest.mark.parametrize("n,bound", [(1, 4), (7, 3), (500, 64), (5000, 1 << 12)])
def test_relabel_first_appearance_matches_dict(gs, n, bound):
    import torch
    rng = np.random.default_rng(n)
    s = rng.integers(0, bound, n)
    d = rng.integers(0, bound, n)
    ts, td = torch.from_numpy(s.copy()), torch.from_numpy(d.copy())
    gs.relabel_first_appearance(ts, td, bound)
    es, ed = _dict_relabel(s, d)
    assert np.array_equal(ts.numpy(), es) and np.array_equal(td.numpy(), ed)


def test_relabel_first_appearance_config4_prefix_is_exact_regime(gs, oracle_mod):
    # the config-4 generator's stream (oracle restatement, small sides) relabelled: the
    # quirk-exact Candidates restatement no longer diverges from the truth
    import torch
    s, d = oracle_mod.bip_edges(0x5EED0B1B, 8, 0, 2000)
    assert oracle_mod.bip_quirk_divergence(s, d)["diverges"]
    ts, td = torch.from_numpy(np.array(s, np.int64)), torch.from_numpy(np.array(d, np.int64))
    gs.relabel_first_appearance(ts, td, 2 << 8)
    assert not oracle_mod.bip_quirk_divergence(ts.numpy(), td.numpy())["diverges"]
