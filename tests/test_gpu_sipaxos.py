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


@pytest.mark.parametrize("P,A,values", [(1, 3, ("a",)), (2, 1, ("a", "b"))])
def test_sipaxos_termination_goal(P, A, values):
    """Goal Termination (every proposer decided): end condition, per-depth counts and goal depth
    equal the oracle's (level-completing rule), and the goal trace replays on the oracle."""
    args = ["--proto", "sipaxos", "--proposers", str(P), "--acceptors", str(A), "--values", ",".join(values),
            "--inv", "Agreement", "--goal", "Termination"]
    want = oracle_util.run("bfs", args + ["--finish-level"], timeout=120)
    proto = SIPaxos(P, A, values)
    s = SearchSettings().addInvariant(proto.predicate("Agreement")).addGoal(proto.predicate("Termination"))
    s.table_log2_slots = 20
    r = Search.bfs(proto.initial_state(), s)
    assert r.endCondition().name == want["end"] == "GOAL_FOUND"
    assert r.per_depth == want["per_depth"]
    st = r.goalMatchingState()
    assert st.depth() == want["terminals"][0]["depth"]
    rep = oracle_util.replay(args, st.trace())
    assert rep["ok"], rep
    assert rep["depth"] == st.depth()
    assert rep["goals"][0]["value"] is True


@pytest.mark.parametrize("shards", [1, 2])
def test_incorrect_sipaxos_agreement_violation(shards):
    """IncorrectSingleInstancePaxos (BadProposer.handleAcceptAck, IncorrectSingleInstancePaxos.java:53-63:
    a decision on acceptAcks * 2 >= acceptors - 1) violates Agreement. Each proposer needs 7 events
    to decide on one AcceptAck (Propose, 2 x Prepare + PrepareAck, Accept + AcceptAck), and the
    second must finish its phase 1 on acceptors that accepted nothing, so the first violation is at
    depth 14. Checked: the levels through 11 equal the oracle's fixture (no violation), the search
    ends INVARIANT_VIOLATED on Agreement at depth 14, and the oracle replays the trace to a state
    that violates Agreement."""
    proto = SIPaxos(2, 3, ("a", "b"), incorrect=True)
    s = SearchSettings().addInvariant(proto.predicate("Integrity")).addInvariant(proto.predicate("Agreement"))
    s.maxDepth(16)
    s.table_log2_slots = 26
    from dslabs_amd import Engine
    e = Engine(proto, virtual_shards=shards if shards > 1 else 0, replicate_below=0 if shards > 1 else -1)
    try:
        r = e.bfs(proto.initial_state(), s)
    finally:
        e.close()
    assert r.endCondition() == EndCondition.INVARIANT_VIOLATED
    assert r.per_depth[:12] == GOLD["sipaxos_incorrect_2p3a"]["per_depth"]
    st = r.invariantViolatingState()
    assert st.depth() == 14 and r.invariantViolated().predicate.name == "Agreement"
    rep = oracle_util.replay(["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b",
                              "--inv", "Integrity", "--inv", "Agreement", "--incorrect"], st.trace())
    assert rep["ok"], rep
    assert rep["depth"] == 14
    assert rep["invariants"][0]["value"] is True and rep["invariants"][1]["value"] is False
