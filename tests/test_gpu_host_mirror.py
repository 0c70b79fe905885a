"""GPU: the reference's own hot-path tests, restated on the C++ host mirror
(tests/cpp/test_reference_suite.cpp -> gelly_streaming.hpp -> libgs_summary.so),
and the ConnectedComponentsExample default stream through the same mirror."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "gelly-streaming_amd", "host", "bin")


def _run(name, *args):
    exe = os.path.join(BIN, name)
    assert os.path.exists(exe), "host mirror not built (run __graft_entry__.build())"
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=120)


def test_reference_suite_on_host_mirror():
    r = _run("test_reference_suite")
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("ConnectedComponentsTest.test", "BipartitenessCheckTest.testBipartite",
                 "BipartitenessCheckTest.testNonBipartite", "DisjointSetTest.testGetMatches",
                 "DisjointSetTest.testFind", "DisjointSetTest.testMerge", "Merger.checkpoint"):
        assert "PASS " + name in r.stdout


def test_connected_components_example_default_stream():
    r = _run("connected_components_example")
    assert r.returncode == 0, r.stderr
    with open(os.path.join(ROOT, "tests", "golden", "derived.json")) as f:
        golden = json.load(f)["cc_default_stream"]["emissions"]
    assert r.stdout.strip().splitlines() == golden
