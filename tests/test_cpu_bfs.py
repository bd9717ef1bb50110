"""The multithreaded CPU baseline (tools/cpu_bfs.cpp, bench.py's cpu_baseline) explores exactly the
oracle's state space: per-depth vectors and end conditions equal the golden fixtures, for any
thread count."""
import json
import os

import pytest

import argmap
from tools import cpu_baseline

HERE = os.path.dirname(os.path.abspath(__file__))


def _gold(fname, name):
    return json.load(open(os.path.join(HERE, "golden", fname + ".json")))[name]


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("fname,name", [("multipaxos", "mp_c5_d8"), ("lab0", "lab0_2c10p_exhaustive"),
                                        ("amokv", "kv_test10_exhaustive"), ("sipaxos", "sipaxos_2p3a_d9"),
                                        ("pb", "pb_2s1c_d15"), ("synthetic", "synth_c3_d5"),
                                        ("multipaxos", "mp_expect_violation"), ("lab0", "lab0_1c10p_goal")])
def test_cpu_bfs_matches_golden(fname, name, threads):
    case = _gold(fname, name)
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto, table_log2=22)
    r = cpu_baseline.run(proto, s, threads=threads)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]
    assert r["states"] == case["states"]
    assert r["threads"] == threads


def test_c3_bench_depth10_fixture_consistent():
    """tests/golden/deep.json synth_c3_d10_cpu_bfs (the host BFS to BASELINE C3's full depth, the
    vector test_gpu_synthetic pins the GPU's bench configuration to) extends the oracle's deepest
    C3 pin and sums to its state count; the same engine reproduces its depth-7 prefix here."""
    deep = json.load(open(os.path.join(HERE, "golden", "deep.json")))
    c = deep["synth_c3_d10_cpu_bfs"]
    assert c["per_depth"][:9] == deep["synth_c3_d8"]["per_depth"]
    assert sum(c["per_depth"]) == c["states"] == 780909037
    assert c["end"] == "SPACE_EXHAUSTED" and c["max_depth"] == 10
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    proto, s, _ = bench.build_search("synthetic", 7)
    r = cpu_baseline.run(proto, s, threads=4, table_log2=24)
    assert r["per_depth"] == c["per_depth"][:8]
