"""lab3 Multi-Paxos (BASELINE C5) on the MI355X engine vs the oracle's golden vectors."""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import EndCondition, Engine, Search

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "multipaxos.json")))


def _run(case, **eng):
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto)
    e = Engine(proto, **eng)
    try:
        return e.bfs(proto.initial_state(), s)
    finally:
        e.close()


@pytest.mark.parametrize("name", sorted(GOLD))
def test_multipaxos_parity(name):
    case = GOLD[name]
    r = _run(case)
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"], name
    assert r.states == case["states"]
    if case["terminal_depth"] >= 0:
        assert r.max_depth == case["terminal_depth"]


@pytest.mark.parametrize("shards,rep", [(2, 0), (8, 0), (8, 2000)])
def test_multipaxos_c5_sharded(shards, rep):
    case = GOLD["mp_c5_d12"]
    r = _run(case, virtual_shards=shards, replicate_below=rep)
    assert r.per_depth == case["per_depth"]


@pytest.mark.parametrize("name", ["mp_expect_violation", "mp_test22_phase1", "mp_singleton"])
def test_multipaxos_trace_replays(name):
    case = GOLD[name]
    r = _run(case)
    st = r.invariantViolatingState() or r.goalMatchingState()
    args = [a for a in case["args"] if a != "--finish-level"]
    rep = oracle_util.replay(args, st.trace())
    assert rep["ok"], rep["error"]
    assert rep["depth"] == st.depth()
    if r.endCondition() == EndCondition.INVARIANT_VIOLATED:
        assert not all(i["value"] for i in rep["invariants"])
    else:
        assert rep["goals"][0]["value"]


def test_test22_two_phase_search():
    """PaxosTest.test22: goal in partition {server1, server2, client1}, then from that state
    CLIENTS_DONE must be reachable in partition {server1, server3, client2}; the second search
    starts from the GPU's own goal state and is checked against the oracle started from the
    same (replayed) state."""
    case = GOLD["mp_test22_phase1"]
    r1 = _run(case)
    assert r1.endCondition() == EndCondition.GOAL_FOUND
    first = r1.goalMatchingState()
    proto = first.protocol
    args2 = ["--proto", "multipaxos", "--workload", "append-xy-expect", "--inv", "RESULTS_OK", "--inv",
             "LOGS_CONSISTENT_ALL_SLOTS", "--goal", "CLIENTS_DONE", "--partition", "server1,server3,client2",
             "--finish-level"]
    r2 = Search.bfs(first, argmap.settings(args2, proto))
    assert r2.endCondition() == EndCondition.GOAL_FOUND
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".trace", delete=False) as f:
        f.write("\n".join(first.trace()) + "\n")
    try:
        want = oracle_util.run("bfs", args2 + ["--start-trace", f.name], timeout=300)
        # the second trace extends the first (the previous chain crosses the start state); its
        # suffix is replayed under the second phase's partition from the first goal state
        full = r2.goalMatchingState().trace()
        assert full[:first.depth()] == first.trace()
        rep = oracle_util.replay(args2[:-1] + ["--start-trace", f.name], full[first.depth():])
    finally:
        os.unlink(f.name)
    # the oracle indexes per_depth by absolute depth (zeros before the start state's depth)
    assert want["per_depth"][:first.depth()] == [0] * first.depth()
    assert r2.per_depth == want["per_depth"][first.depth():]
    assert r2.initial_depth == first.depth()
    assert rep["ok"] and rep["goals"][0]["value"], rep
    assert rep["depth"] == r2.goalMatchingState().depth()


# PaxosTest.test27 (PaxosTest.java:1214-1228): singleton Paxos, putAppendGetWorkload; the goal
# CLIENTS_DONE is reached at depth exactly 6, then the space with CLIENTS_DONE pruned is exhausted.
# lab3 predicates (PaxosTest.java:113-346) and StatePredicate combinators (:397-431).
LIVE = {
    "test27_goal": ["--proto", "multipaxos", "--servers", "1", "--clients", "1", "--workload", "put-append-get",
                    "--inv", "RESULTS_OK", "--goal", "CLIENTS_DONE", "--max-depth", "6"],
    "test27_exhaustive": ["--proto", "multipaxos", "--servers", "1", "--clients", "1", "--workload",
                          "put-append-get", "--inv", "RESULTS_OK", "--prune", "CLIENTS_DONE"],
    "goal_has_status": ["--proto", "multipaxos", "--workload", "append-xy", "--inv", "RESULTS_OK", "--inv",
                        "LOGS_CONSISTENT", "--goal", "hasStatus:server2:1:CHOSEN", "--max-depth", "10"],
    "inv_implies": ["--proto", "multipaxos", "--workload", "append-xy", "--inv",
                    "implies(hasStatus:server1:1:CHOSEN,hasCommand:server1:1:X)", "--inv", "slotValid:1",
                    "--max-depth", "10"],
    "goal_and_or": ["--proto", "multipaxos", "--workload", "append-xy", "--inv", "LOGS_CONSISTENT_ALL_SLOTS",
                    "--goal", "and(hasStatus:server1:2:CHOSEN,or(hasStatus:server2:2:ACCEPTED,"
                    "!hasStatus:server3:2:EMPTY))", "--max-depth", "9"],
    "c5_lab3_invariants": ["--proto", "multipaxos", "--workload", "append-xy", "--inv", "RESULTS_OK", "--inv",
                           "LOGS_CONSISTENT", "--inv", "and(slotValid:1,slotValid:2)", "--inv",
                           "APPENDS_LINEARIZABLE", "--max-depth", "10"],
}


@pytest.mark.parametrize("name", sorted(LIVE))
def test_multipaxos_lab3_predicates_and_test27(name):
    args = LIVE[name]
    want = oracle_util.run("bfs", args + ["--finish-level"], timeout=300)
    proto = argmap.protocol(args)
    r = Search.bfs(proto.initial_state(), argmap.settings(args, proto))
    assert r.endCondition().name == want["end"]
    assert r.per_depth == want["per_depth"]
    st = r.invariantViolatingState() or r.goalMatchingState()
    if name == "test27_goal":
        assert r.endCondition() == EndCondition.GOAL_FOUND and st.depth() == 6
    if st is not None:
        rep = oracle_util.replay(args, st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth()
        if r.endCondition() == EndCondition.INVARIANT_VIOLATED:
            assert not all(i["value"] for i in rep["invariants"])
        else:
            assert rep["goals"][0]["value"]
