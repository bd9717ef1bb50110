"""Queued levels (BfsEngine::enqueue_queue) against one launch per level and the golden vectors.

A queue runs several levels without a host round trip and stops where the host must act: spilled
rows, a terminal, an error, a frontier past its capacity. DSL_QUEUE_ROWS forces tiny queues so
every stop reason is taken mid-queue; DSL_NO_QUEUE turns the queue off. Results must not move.
"""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import Engine

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _gold(fname, name):
    return json.load(open(os.path.join(HERE, "golden", fname + ".json")))[name]


CASES = [("multipaxos", "mp_c5_d8"), ("multipaxos", "mp_expect_violation"), ("multipaxos", "mp_test22_phase1"),
         ("lab0", "lab0_2c10p_exhaustive"), ("lab0", "lab0_1c10p_goal"), ("synthetic", "synth_3n_k8_d9"),
         ("amokv", "kv_test09_goal"), ("pb", "pb_2s1c_d15"), ("pb", "pb_2c_results_violation")]
MODES = [{}, {"DSL_NO_QUEUE": "1"}, {"DSL_QUEUE_ROWS": "64"}, {"DSL_QUEUE_ROWS": "2048"}]


@pytest.mark.parametrize("mode", MODES, ids=lambda m: ",".join("%s=%s" % kv for kv in m.items()) or "default")
@pytest.mark.parametrize("fname,name", CASES)
def test_queue_modes_match_golden(fname, name, mode, monkeypatch):
    for k, v in mode.items():
        monkeypatch.setenv(k, v)
    case = _gold(fname, name)
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto)
    e = Engine(proto)
    try:
        for _ in range(2):  # the second run reuses the engine's buffers and queue size
            r = e.bfs(proto.initial_state(), s)
            assert r.endCondition().name == case["end"]
            assert r.per_depth == case["per_depth"]
            assert r.states == case["states"]
            st = r.invariantViolatingState() or r.goalMatchingState()
            if st is not None:
                args = [a for a in case["args"] if a != "--finish-level"]
                rep = oracle_util.replay(args, st.trace())
                assert rep["ok"], rep["error"]
                assert rep["depth"] == st.depth()
    finally:
        e.close()


@pytest.mark.parametrize("secs", [0.005, 0.02])
def test_time_limit_ends_queued_search(secs):
    """SearchSettings.maxTimeSecs (Search.java:127-133, :313-318): an unbounded C5 search ends
    TIME_EXHAUSTED soon after the limit, also inside a level (every workgroup checks the device-side
    deadline before each chunk) and when queued levels are running; the levels it completed match
    the golden vector (a level the deadline cut short is not a completed depth)."""
    case = _gold("multipaxos", "mp_c5_d12")
    args = [a for a in case["args"]]
    k = args.index("--max-depth")
    del args[k:k + 2]
    proto = argmap.protocol(args)
    s = argmap.settings(args, proto, table_log2=27)
    s.maxTimeSecs(secs)
    e = Engine(proto)
    try:
        # the queued levels' kernels load on their first launch (ms): a depth-8 search without a
        # limit first, so that a test run alone times the same warm engine as the whole suite does
        warm = argmap.settings(case["args"][:k] + ["--max-depth", "8"] + case["args"][k + 2:], proto, table_log2=27)
        pd = e.bfs(proto.initial_state(), warm).per_depth
        assert len(pd) >= 8 and pd == case["per_depth"][:len(pd)], pd
        for run in range(4):  # the first run also allocates the table; later ones have a queue time
            r = e.bfs(proto.initial_state(), s)
            assert r.endCondition().name == "TIME_EXHAUSTED"
            # the first run allocates the 1 GiB table and the level buffers (hipMalloc, slow and
            # variable); the second, with the whole limit for levels, reaches deeper and sizes the
            # queue's history levels for that span (GiBs of hipMalloc, once: a 1.8 s outlier on
            # one box); later runs allocate nothing and stop right after the limit (a level past
            # the deadline stops at its next chunk)
            print(f"time limit {secs}: run {run} {r.elapsed_s:.4f} s, depth {len(r.per_depth)}")
            assert r.elapsed_s < secs + (2.5 if run < 2 else 0.25), (run, r.elapsed_s)
            n = min(len(r.per_depth), len(case["per_depth"]))
            assert r.per_depth[:n] == case["per_depth"][:n]
            if run:
                assert n >= 6, r.per_depth
    finally:
        e.close()


def test_do_checks_determinism_and_idempotence():
    """GlobalSettings.doErrorChecks / doAllChecks (Search.java:201-220, CheckLogger.java:104-121):
    every level's sampled new states re-derived on the host equal the device's rows (C5 d8, no
    non-determinism); the synthetic protocol's Poke handler (pokes + 1 mod 4) is not idempotent and
    is reported, Multi-Paxos's handlers are; a corrupted row (DSL_CHECK_FLIP) is reported as not
    deterministic. Per-depth counts are unchanged by the checks."""
    import json
    import os
    import sys
    import argmap
    from dslabs_amd import Engine
    HERE = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(HERE))
    import bench
    case = json.load(open(os.path.join(HERE, "golden", "multipaxos.json")))["mp_c5_d12"]
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto, table_log2=22).doAllChecks()
    s.maxDepth(8)
    e = Engine(proto)
    try:
        r = e.bfs(proto.initial_state(), s)
    finally:
        e.close()
    assert r.per_depth == case["per_depth"][:9]
    assert r.checks["run"] > 500 and r.checks["not_deterministic"] == 0 and r.checks["not_idempotent"] == 0, r.checks
    sp, ss, _ = bench.build_search("synthetic", 5)
    ss.table_log2_slots = 22
    ss.doAllChecks()
    e = Engine(sp)
    try:
        r = e.bfs(sp.initial_state(), ss)
        assert r.checks["not_deterministic"] == 0 and r.checks["not_idempotent"] > 0, r.checks
        assert "Poke" in r.checks["first_not_idempotent"], r.checks
        ss.doErrorChecks()
        os.environ["DSL_CHECK_FLIP"] = "1"
        try:
            r = e.bfs(sp.initial_state(), ss)
        finally:
            del os.environ["DSL_CHECK_FLIP"]
        assert r.checks["not_deterministic"] >= 1 and r.checks["not_idempotent"] == 0, r.checks
    finally:
        e.close()
