"""Random depth-first search (Search.dfs / RandomDFS, Search.java:397-402, :507-583) on the device:
probes find the reference's known violations and goals, every reported trace replays on the oracle
and ends in a state with the reported predicate value, and a space without terminals ends
TIME_EXHAUSTED (RandomDFS never exhausts a space)."""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import CLIENTS_DONE, RESULTS_OK, EndCondition, Engine, SearchSettings
from dslabs_amd.protocols import PingPong

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
LAB0 = json.load(open(os.path.join(HERE, "golden", "lab0.json")))
MP = json.load(open(os.path.join(HERE, "golden", "multipaxos.json")))
SYN = json.load(open(os.path.join(HERE, "golden", "synthetic.json")))


def _dfs(case_args, max_depth, **kw):
    proto = argmap.protocol(case_args)
    s = argmap.settings(case_args, proto)
    s.maxDepth(max_depth)
    s.maxTimeSecs(60)
    e = Engine(proto)
    try:
        return e.dfs(proto.initial_state(), s, **kw)
    finally:
        e.close()


def _replay_ok(case_args, st, end):
    args = [a for a in case_args if a != "--finish-level"]
    rep = oracle_util.replay(args, st.trace())
    assert rep["ok"], rep["error"]
    assert rep["depth"] == st.depth()
    if end == EndCondition.INVARIANT_VIOLATED:
        assert not all(i["value"] and not i["threw"] for i in rep["invariants"])
    else:
        assert any(g["value"] for g in rep["goals"])


@pytest.mark.parametrize("name,fixture,depth", [
    ("lab0_mutant_nocheck", LAB0, 30),           # README "When Things Go Wrong": RESULTS_OK violated
    ("mp_expect_violation", MP, 14),             # Multi-Paxos, client2 ordered first: RESULTS_OK violated
    ("synth_counter_violation", SYN, 12),        # synthetic: a node value reaches the bound
])
def test_dfs_finds_violation_and_trace_replays(name, fixture, depth):
    case = fixture[name]
    r = _dfs(case["args"], depth, probes=16384, seed=7)
    assert r.endCondition() == EndCondition.INVARIANT_VIOLATED, r.endCondition()
    st = r.invariantViolatingState()
    assert st.depth() >= case["terminal_depth"]  # BFS depth is the minimum
    _replay_ok(case["args"], st, EndCondition.INVARIANT_VIOLATED)


def test_dfs_goal():
    # 2 pings (the README's state graph, goal at depth 4): random walks revisit old messages, so
    # a deep goal (10 pings) is rarely hit within a depth bound -- as for the JVM's RandomDFS
    case = LAB0["lab0_1c2p_goal"]
    r = _dfs(case["args"], 12, probes=4096, seed=3)
    assert r.endCondition() == EndCondition.GOAL_FOUND
    st = r.goalMatchingState()
    assert st.depth() >= 4
    _replay_ok(case["args"], st, EndCondition.GOAL_FOUND)


def test_dfs_without_terminal_runs_out_of_budget():
    proto = PingPong(1, 10)
    s = SearchSettings().addInvariant(RESULTS_OK).addPrune(CLIENTS_DONE)
    s.maxDepth(40)
    e = Engine(proto)
    try:
        r = e.dfs(proto.initial_state(), s, probes=4096, seed=1, max_probes=20000)
    finally:
        e.close()
    assert r.endCondition() == EndCondition.TIME_EXHAUSTED
    assert r.states >= 20000  # every probe counts its initial state, plus each successor


@pytest.mark.parametrize("name,fixture,max_trace", [
    ("lab0_mutant_nocheck", LAB0, 5),
    ("synth_counter_violation", SYN, None),
])
def test_dfs_unbounded_depth_small_trace_capacity(name, fixture, max_trace):
    """No maxDepth: probes run until they reach max_trace events and are then restarted before
    stepping, so a reported terminal is always within the recorded trace; the trace replays on
    the oracle to a state with the reported predicate value (depth = trace length)."""
    case = fixture[name]
    cap = max_trace or case["terminal_depth"] + 2
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto)
    s.maxTimeSecs(60)
    e = Engine(proto)
    try:
        r = e.dfs(proto.initial_state(), s, probes=16384, seed=11, max_trace=cap, minimize=False)
    finally:
        e.close()
    assert r.endCondition() == EndCondition.INVARIANT_VIOLATED, r.endCondition()
    st = r.invariantViolatingState()
    assert case["terminal_depth"] <= st.depth() <= cap
    assert len(st.trace()) == st.depth()
    _replay_ok(case["args"], st, EndCondition.INVARIANT_VIOLATED)
