"""Regenerate the committed golden fixtures in tests/golden/.

  reference_pins.json  -- inputs/outputs held by the reference's own tests
                          (data transcribed from ConnectedComponentsTest.java:41,54-63,
                          BipartitenessCheckTest.java:40-42,63-65,71-91,
                          DisjointSetTest.java:37-77). Written by hand below.
  derived.json         -- outputs of the oracle (oracle/gs_oracle.cpp) on the two
                          bundled default streams (ConnectedComponentsExample.java:121-139,
                          BipartitenessCheckExample.java:109-118), each cross-checked here
                          against an independent networkx computation.
  streams.npz          -- prefixes of the synthetic stream spec (RMAT / ER / bipartite)
                          plus canonical CC labels of small streams, cross-checked
                          against networkx.

Run: python tests/golden/make_golden.py   (CPU only; needs networkx, present here)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

PINS = {
    "cc_test": {
        "source": "src/test/java/org/apache/flink/graph/streaming/example/test/ConnectedComponentsTest.java:41,54-63",
        "edges": [[1, 2], [1, 3], [2, 3], [1, 5], [6, 7], [8, 9]],
        "window_ms": 5,
        "expected_lines": ["1, 2, 3, 5", "6, 7", "8, 9"],
    },
    "bip_test_bipartite": {
        "source": "src/test/java/org/apache/flink/graph/streaming/example/test/BipartitenessCheckTest.java:40-42,71-80",
        "edges": [[1, 2], [1, 3], [1, 4], [4, 5], [4, 7], [4, 9]],
        "window_ms": 500,
        "expected": ["(true,{1={1=(1,true), 2=(2,false), 3=(3,false), 4=(4,false), 5=(5,true), 7=(7,true), 9=(9,true)}})"],
    },
    "bip_test_non_bipartite": {
        "source": "src/test/java/org/apache/flink/graph/streaming/example/test/BipartitenessCheckTest.java:63-65,82-91",
        "edges": [[1, 2], [2, 3], [3, 1], [4, 5], [5, 7], [4, 1]],
        "window_ms": 500,
        "expected": ["(false,{})"],
    },
    "disjointset_test": {
        "source": "src/test/java/org/apache/flink/graph/streaming/util/DisjointSetTest.java:37-77",
        "setup_unions": [[i, i + 2] for i in range(8)],
        "expected_matches": 10,
        "merge_unions": [[i, i + 100] for i in range(8)],
        "expected_matches_after_merge": 18,
        "expected_roots_after_merge": 2,
    },
}


def nx_components(src, dst):
    import networkx as nx
    g = nx.Graph()
    for a, b in zip(src, dst):
        g.add_edge(int(a), int(b))
    lab = {}
    for comp in nx.connected_components(g):
        m = min(comp)
        for v in comp:
            lab[v] = m
    return lab


def main():
    with open(os.path.join(HERE, "reference_pins.json"), "w") as f:
        json.dump(PINS, f, indent=1)

    derived = {}
    # CC default stream: edges (k, k+2), event time 100k ms, 1000 ms windows.
    k = np.arange(1, 101, dtype=np.int64)
    win = (k * 100) // 1000
    em = oracle.cc_dataflow(k, k + 2, win)
    # independent check of every window's cumulative result
    for wi, w in enumerate(sorted(set(win.tolist()))):
        m = win <= w
        lab = nx_components(k[m], (k + 2)[m])
        v = np.array(sorted(lab), dtype=np.int64)
        assert oracle.canonical_cc_string(v, [lab[x] for x in v.tolist()]) == em[wi]
    derived["cc_default_stream"] = {
        "source": "src/main/java/org/apache/flink/graph/streaming/example/ConnectedComponentsExample.java:121-139",
        "edges": "k -> (k, k+2), k = 1..100, timestamp 100*k ms",
        "window_ms": 1000,
        "emissions": em,
    }
    # Bipartite default stream: (k, 2k+1) x10 for k = 1..100, one window.
    kk = np.repeat(np.arange(1, 101, dtype=np.int64), 10)
    bem = oracle.bip_dataflow(kk, 2 * kk + 1)
    ok, comp, v, sign = oracle.bip_truth(kk, 2 * kk + 1)
    assert bem == [oracle.canonical_candidates_string(ok, comp, v, sign)]
    derived["bip_default_stream"] = {
        "source": "src/main/java/org/apache/flink/graph/streaming/example/BipartitenessCheckExample.java:109-118",
        "edges": "k -> 10 x (k, 2k+1), k = 1..100, one window",
        "emissions": bem,
    }
    # Order quirk of Candidates.merge: same triangle, two orders.
    derived["bip_triangle_quirk"] = {
        "order_231": oracle.bip_dataflow([2, 1, 1], [3, 2, 3]),
        "order_123": oracle.bip_dataflow([1, 2, 1], [2, 3, 3]),
    }
    with open(os.path.join(HERE, "derived.json"), "w") as f:
        json.dump(derived, f, indent=1)

    arrays = {}
    s, d = oracle.rmat_edges(0x5EED0020, 20, 0, 4096, True)
    arrays["rmat20_prefix_src"], arrays["rmat20_prefix_dst"] = s, d
    s, d = oracle.rmat_edges(0x5EED0026, 26, (1 << 29) - 2048, 4096, True)
    arrays["rmat26_mid_src"], arrays["rmat26_mid_dst"] = s, d
    s, d = oracle.er_edges(0x5EED00E5, 22, 0, 4096, True)
    arrays["er22_prefix_src"], arrays["er22_prefix_dst"] = s, d
    inj = [100, 1000, 3000]
    s, d = oracle.bip_edges(0x5EED0B1B, 19, 0, 4096, inj)
    arrays["bip19_prefix_src"], arrays["bip19_prefix_dst"] = s, d
    arrays["bip19_prefix_inject"] = np.array(inj, dtype=np.uint64)
    # small RMAT stream with canonical labels (oracle == networkx)
    s, d = oracle.rmat_edges(0x5EED0012, 12, 0, 1 << 14, True)
    v, lab = oracle.cc_labels(s, d)
    ref = nx_components(s, d)
    assert [ref[x] for x in v.tolist()] == lab.tolist()
    arrays["rmat12_src"], arrays["rmat12_dst"] = s, d
    arrays["rmat12_v"], arrays["rmat12_label"] = v, lab
    np.savez_compressed(os.path.join(HERE, "streams.npz"), **arrays)
    print("golden fixtures written")


if __name__ == "__main__":
    main()
