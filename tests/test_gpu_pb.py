"""lab2 primary-backup + ViewServer (BASELINE C4) on the MI355X engine vs the
oracle's golden vectors: per-depth counts, end conditions, replayable traces, sharding."""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import Engine

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pb.json")))


def _run(case, **eng):
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto)
    e = Engine(proto, **eng)
    try:
        return e.bfs(proto.initial_state(), s)
    finally:
        e.close()


@pytest.mark.parametrize("name", sorted(GOLD))
def test_pb_parity(name):
    case = GOLD[name]
    r = _run(case)
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"], name
    assert r.states == case["states"]
    if case["terminal_depth"] >= 0:
        assert r.max_depth == case["terminal_depth"]
        st = r.invariantViolatingState() or r.goalMatchingState()
        args = [a for a in case["args"] if a != "--finish-level"]
        rep = oracle_util.replay(args, st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth() == case["terminal_depth"]


@pytest.mark.parametrize("shards,rep", [(2, 0), (3, 0), (4, 2000)])
def test_pb_sharded(shards, rep):
    case = GOLD["pb_2s2c_d11"]
    r = _run(case, virtual_shards=shards, replicate_below=rep)
    assert r.per_depth == case["per_depth"]
