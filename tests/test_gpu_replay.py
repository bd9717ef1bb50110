"""Trace replay (dsl_replay: TraceReplaySearch) and trace minimization (TraceMinimizer, as
RandomDFS applies it) on the engine's transition functions, against the reference's own
minimizer tests and against the oracle's restatement of TraceMinimizer on the same raw traces."""
import json
import os

import pytest

import argmap
import oracle_util
from test_oracle_golden import MINI_CASES
from dslabs_amd import EndCondition, Engine

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _gold(fname, name):
    return json.load(open(os.path.join(HERE, "golden", fname + ".json")))[name]


def _mini_event(proto, line):
    # "Message(a -> b, Foo())"
    body = line[len("Message("):-1]
    route, msg = body.split(", ", 1)
    frm, to = route.split(" -> ")
    return proto.event(frm, to, msg[:-2])


@pytest.mark.parametrize("case", MINI_CASES, ids=[c[0] for c in MINI_CASES])
def test_replay_minimizes_like_the_reference(case):
    """SearchAndTraceMinimizerTest: depth 3 replayed as is, depth 2 once minimized."""
    _, sargs, trace, end, dmin, draw = case
    args = ["--proto", "minitest"] + sargs
    proto = argmap.protocol(args)
    s = argmap.settings(args, proto)
    events = [_mini_event(proto, line) for line in trace]
    e = Engine(proto)
    try:
        for minimize, depth in ((True, dmin), (False, draw)):
            r = e.replay(proto.initial_state(), s, events, minimize)
            assert r.endCondition().name == end
            assert r.max_depth == depth
            want = oracle_util.replay_search(args, trace, minimize)
            st = r.invariantViolatingState() or r.goalMatchingState() or r.exceptionalState()
            if end == "SPACE_EXHAUSTED":
                assert st is None
            else:
                assert st.depth() == depth
                assert st.trace() == want["trace"]
    finally:
        e.close()


def test_replay_stops_at_an_undeliverable_event():
    args = ["--proto", "minitest", "--inv", "foo"]
    proto = argmap.protocol(args)
    s = argmap.settings(args, proto)
    # Bar from b is not in the network before b handled a Foo
    events = [proto.event("b", "a", "Bar"), proto.event("a", "b", "Foo")]
    e = Engine(proto)
    try:
        r = e.replay(proto.initial_state(), s, events, True)
    finally:
        e.close()
    assert r.endCondition() == EndCondition.SPACE_EXHAUSTED
    assert r.max_depth == 0


DFS_CASES = [("lab0", "lab0_mutant_nocheck", 30), ("multipaxos", "mp_expect_violation", 14),
             ("synthetic", "synth_counter_violation", 12), ("pb", "pb_2c_results_violation", 16),
             ("amokv", "kv_getput_2c", 12)]


@pytest.mark.parametrize("fname,name,depth", DFS_CASES)
def test_dfs_minimization_matches_oracle_minimizer(fname, name, depth):
    case = _gold(fname, name)
    args = [a for a in case["args"] if a != "--finish-level"]
    proto = argmap.protocol(args)
    s = argmap.settings(args, proto)
    s.maxDepth(depth)
    s.maxTimeSecs(60)
    e = Engine(proto)
    try:
        raw = e.dfs(proto.initial_state(), s, probes=8192, seed=11, minimize=False)
        assert raw.endCondition() == EndCondition.INVARIANT_VIOLATED
        st = raw.invariantViolatingState()
        # the engine's minimizer on the probe's raw trace, against the oracle's on the same trace
        want = oracle_util.replay_search(args, st.trace(), True)
        got = e.replay(proto.initial_state(), s, st.events(), True)
        assert got.endCondition().name == want["end"] == "INVARIANT_VIOLATED"
        mst = got.invariantViolatingState()
        assert mst.trace() == want["trace"]
        assert mst.depth() == want["depth"] <= st.depth()
        assert mst.depth() >= case["terminal_depth"]  # BFS depth is the minimum
        # a minimizing DFS reports a trace that the oracle's minimizer leaves unchanged
        mini = e.dfs(proto.initial_state(), s, probes=8192, seed=11)
        mt = mini.invariantViolatingState()
        again = oracle_util.replay_search(args, mt.trace(), True)
        assert again["trace"] == mt.trace()
    finally:
        e.close()


@pytest.mark.parametrize("fname,name,depth", DFS_CASES)
def test_human_readable_trace_matches_oracle(fname, name, depth):
    """SearchState.humanReadableTrace on raw random-DFS traces (long, with no-op steps): the
    engine's reordering equals the oracle's and ends in the same state."""
    case = _gold(fname, name)
    args = [a for a in case["args"] if a != "--finish-level"]
    proto = argmap.protocol(args)
    s = argmap.settings(args, proto)
    s.maxDepth(depth)
    s.maxTimeSecs(60)
    e = Engine(proto)
    try:
        raw = e.dfs(proto.initial_state(), s, probes=8192, seed=5, minimize=False)
        st = raw.invariantViolatingState()
        hr = e.human_readable_trace(proto.initial_state(), s, st.events())
        want = oracle_util.replay_search(args + ["--human-readable"], st.trace(), False)
        assert want["end"] == "INVARIANT_VIOLATED"  # the raw trace replays to its violation
        assert hr.trace() == want["trace"]
        assert hr.depth() == want["depth"] == len(want["trace"]) <= st.depth()
        assert hr.packed == st.packed  # same end state
    finally:
        e.close()
