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
