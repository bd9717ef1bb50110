"""lab0 PingPong on the MI355X engine vs the oracle's golden vectors (bit-exact per depth)."""
import json
import os

import pytest

import oracle_util
from dslabs_amd import (CLIENTS_DONE, RESULTS_OK, EndCondition, Search, SearchSettings, clientDone)
from dslabs_amd.protocols import PingPong

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "lab0.json")))


def settings_from_args(args):
    """Builds SearchSettings from oracle CLI args (same meaning)."""
    s = SearchSettings()
    s.table_log2_slots = 22
    named = {"RESULTS_OK": RESULTS_OK, "CLIENTS_DONE": CLIENTS_DONE}
    it = iter(range(len(args)))
    i = 0
    while i < len(args):
        a = args[i]
        v = args[i + 1] if i + 1 < len(args) else None
        if a == "--inv":
            s.addInvariant(named[v]); i += 1
        elif a == "--goal":
            s.addGoal(named[v]); i += 1
        elif a == "--prune":
            s.addPrune(named[v]); i += 1
        elif a == "--max-depth":
            s.maxDepth(int(v)); i += 1
        elif a == "--no-timers":
            s.deliverTimers(v, False); i += 1
        elif a == "--partition":
            s.partition(*[g.split(",") for g in v.split("|")]); i += 1
        i += 1
    return s


def proto_from_args(args):
    d = dict(zip(args[::1], args[1::1]))
    clients = int(args[args.index("--clients") + 1])
    pings = int(args[args.index("--pings") + 1])
    return PingPong(clients, pings, check_value="--mutant-no-check" not in args,
                    reset_timer="--mutant-no-reset" not in args)


@pytest.mark.parametrize("name", sorted(GOLD))
def test_lab0_parity(name):
    case = GOLD[name]
    proto = proto_from_args(case["args"])
    r = Search.bfs(proto.initial_state(), settings_from_args(case["args"]))
    assert r.endCondition().name == case["end"]
    if case["terminal_depth"] >= 0:
        # level-synchronous rule: compare all complete levels; the terminal level is complete
        # only in --finish-level fixtures
        assert r.max_depth == case["terminal_depth"]
        full = "--finish-level" in case["args"]
        n = len(case["per_depth"]) if full else len(case["per_depth"]) - 1
        assert r.per_depth[:n] == case["per_depth"][:n]
        if full:
            assert r.states == case["states"]
    else:
        assert r.per_depth == case["per_depth"]
        assert r.states == case["states"]
        assert r.max_depth == case["max_depth"]


def test_readme_mutant_trace_replays_on_oracle():
    """Trace of the GPU counterexample is minimal (depth 3) and replays on the oracle."""
    case = GOLD["lab0_mutant_nocheck"]
    proto = PingPong(1, 10, check_value=False)
    s = SearchSettings().addInvariant(RESULTS_OK).addGoal(CLIENTS_DONE)
    r = Search.bfs(proto.initial_state(), s)
    assert r.endCondition() == EndCondition.INVARIANT_VIOLATED
    st = r.invariantViolatingState()
    assert st.depth() == 3
    assert st.trace() == case["pinned"]["trace"]
    args = [a for a in case["args"] if a != "--finish-level"]
    rep = oracle_util.replay(args, st.trace())
    assert rep["ok"] and rep["invariants"][0]["value"] is False
    assert r.invariantViolated().predicate is RESULTS_OK


def test_goal_then_restart_from_goal_state():
    """bfs(goal state of an earlier search) like PaxosTest.java:898-910: depth carries over."""
    proto = PingPong(1, 3)
    s = SearchSettings().addInvariant(RESULTS_OK).addGoal(clientDone("client1").negate().negate())
    s.table_log2_slots = 20
    r = Search.bfs(proto.initial_state(), s)
    assert r.endCondition() == EndCondition.GOAL_FOUND
    g = r.goalMatchingState()
    s2 = SearchSettings().addInvariant(RESULTS_OK)
    s2.table_log2_slots = 20
    r2 = Search.bfs(g, s2)
    assert r2.endCondition() == EndCondition.SPACE_EXHAUSTED
    assert r2.initial_depth == g.depth()
    assert r2.per_depth[0] == 1


def test_time_limit_reports_time_exhausted():
    proto = PingPong(2, 10)
    s = SearchSettings().addInvariant(RESULTS_OK).addPrune(CLIENTS_DONE).maxTimeSecs(1)
    s.table_log2_slots = 22
    r = Search.bfs(proto.initial_state(), s)
    assert r.endCondition() in (EndCondition.SPACE_EXHAUSTED, EndCondition.TIME_EXHAUSTED)
