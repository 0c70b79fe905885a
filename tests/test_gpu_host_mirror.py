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


def _run(name, *args, env=None):
    exe = os.path.join(BIN, name)
    assert os.path.exists(exe), "host mirror not built (run __graft_entry__.build())"
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=120, env=env)


def test_reference_suite_on_host_mirror():
    r = _run("test_reference_suite")
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("ConnectedComponentsTest.test", "BipartitenessCheckTest.testBipartite",
                 "BipartitenessCheckTest.testNonBipartite", "DisjointSetTest.testGetMatches",
                 "DisjointSetTest.testFind", "DisjointSetTest.testMerge", "Merger.checkpoint",
                 "windows.negative_extreme"):
        assert "PASS " + name in r.stdout


def test_reference_suite_under_host_sanitizers():
    """the same suite with AddressSanitizer + UBSan on the host code
    (the C++ mirror, the ABI's host side as the test drives it; device code untouched,
    host/Makefile bin/test_reference_suite_san). Any report fails the run."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = _run("test_reference_suite_san", env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failure(s)" in r.stdout and r.stdout.count("PASS ") >= 9, r.stdout
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]


def test_connected_components_example_default_stream():
    r = _run("connected_components_example")
    assert r.returncode == 0, r.stderr
    with open(os.path.join(ROOT, "tests", "golden", "derived.json")) as f:
        golden = json.load(f)["cc_default_stream"]["emissions"]
    assert r.stdout.strip().splitlines() == golden
