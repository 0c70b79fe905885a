import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def gs():
    import gsamd
    gsamd.lib()  # fails loudly if the HIP library is missing
    return gsamd


@pytest.fixture
def fake_comm(gs):
    """Groups created in the test run their collectives through the in-process emulation
    (gs_group_set_comm_api; tests/cpp/gs_fake_comm.cpp), which also fails any collective
    whose ranks issued the communicators' collectives in different orders."""
    gs.use_comm_emulation(True)
    gs.fake_comm().gs_fake_comm_last_error()  # clear
    yield gs
    gs.use_comm_emulation(False)
    err = gs.fake_comm().gs_fake_comm_last_error()
    assert err == 0, "comm emulation error %d (collective order or size)" % err


@pytest.fixture
def knobs(gs):
    """Set include/gs_testing.h knobs for one test: knobs(group_self_apply=1). Restored after."""
    names = set()

    def setk(**kw):
        for k, v in kw.items():
            gs.testing_set(k, v)
            names.add(k)
    yield setk
    for k in names:
        gs.testing_set(k, None)
