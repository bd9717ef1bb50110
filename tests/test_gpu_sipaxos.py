"""Single-instance Paxos (the reference's only complete Paxos) on the MI355X engine vs oracle."""
import json
import os

import pytest

import oracle_util
from dslabs_amd import EndCondition, Search, SearchSettings
from dslabs_amd.protocols import SIPaxos

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sipaxos.json")))


def _settings(proto, depth):
    s = SearchSettings().addInvariant(proto.predicate("Integrity")).addInvariant(proto.predicate("Agreement"))
    s.maxDepth(depth)
    s.table_log2_slots = 24
    return s


@pytest.mark.parametrize("name,P,A,values,incorrect,depth", [
    ("sipaxos_2p3a_d9", 2, 3, ("a", "b"), False, 9),
    ("sipaxos_2p3a_d6", 2, 3, ("a", "b"), False, 6),
    ("sipaxos_3p3a_d6", 3, 3, ("a", "b", "c"), False, 6),
    ("sipaxos_incorrect_2p3a", 2, 3, ("a", "b"), True, 11),
])
def test_sipaxos_parity(name, P, A, values, incorrect, depth):
    proto = SIPaxos(P, A, values, incorrect)
    r = Search.bfs(proto.initial_state(), _settings(proto, depth))
    assert r.endCondition() == EndCondition.SPACE_EXHAUSTED
    assert r.per_depth == GOLD[name]["per_depth"]


def test_sipaxos_goal_trace_replays():
    """Goal "one proposer decided" via negated predicate; trace replays on the oracle."""
    proto = SIPaxos(2, 3, ("a", "b"))
    s = SearchSettings().addInvariant(proto.predicate("Agreement")).addGoal(proto.predicate("Termination"))
    s.maxDepth(14)
    s.table_log2_slots = 26
    r = Search.bfs(proto.initial_state(), s)
    if r.endCondition() != EndCondition.GOAL_FOUND:
        pytest.skip("Termination not reachable within depth 14")
    st = r.goalMatchingState()
    rep = oracle_util.replay(["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b",
                              "--inv", "Agreement", "--goal", "Termination"], st.trace())
    assert rep["ok"], rep
    assert rep["depth"] == st.depth()
    assert rep["goals"][0]["value"] is True
