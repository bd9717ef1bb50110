"""The IR-generated PingPong (dslabs_amd/ir/specs/pingpong.py -> csrc/protocols/gen/pingpong_ir.hpp)
on the MI355X engine: the hand-written protocol's golden vectors, and counterexample traces that
replay on the IR-generated oracle form."""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import EndCondition, Engine

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
LAB0 = json.load(open(os.path.join(HERE, "golden", "lab0.json")))
NAMES = sorted(n for n in LAB0 if "--finish-level" in LAB0[n]["args"] or LAB0[n]["end"] == "SPACE_EXHAUSTED")


def _ir(args):
    return ["pingpong_ir" if a == "pingpong" else a for a in args]


@pytest.mark.parametrize("shards", [0, 3])
@pytest.mark.parametrize("name", NAMES)
def test_ir_pingpong_matches_golden(name, shards):
    case = LAB0[name]
    args = _ir(case["args"])
    proto = argmap.protocol(args)
    e = Engine(proto, virtual_shards=shards, replicate_below=0 if shards else -1)
    try:
        r = e.bfs(proto.initial_state(), argmap.settings(args, proto, table_log2=20))
    finally:
        e.close()
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"]
    st = r.invariantViolatingState() or r.goalMatchingState()
    if st is not None:
        rep = oracle_util.replay([a for a in args if a != "--finish-level"], st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth()
        if r.endCondition() == EndCondition.INVARIANT_VIOLATED:
            assert not all(i["value"] for i in rep["invariants"])


KV = json.load(open(os.path.join(HERE, "golden", "amokv.json")))
KV_NAMES = sorted(n for n in KV if "APPENDS_LINEARIZABLE" not in KV[n]["args"])


@pytest.mark.parametrize("name", KV_NAMES)
def test_ir_amokv_matches_golden(name):
    """The IR-generated AMO-KV (dslabs_amd/ir/specs/amokv.py) against the hand-written
    protocol's golden vectors; traces replay on the IR-generated oracle form."""
    from test_ir import _kv_ir
    case = KV[name]
    proto, rest = _kv_ir(case["args"])
    r = Engine(proto).bfs(proto.initial_state(), argmap.settings(rest, proto, table_log2=22))
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"]
    st = r.invariantViolatingState() or r.goalMatchingState()
    if st is not None:
        rep = oracle_util.replay(proto.oracle_args() + [a for a in rest if a != "--finish-level"], st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth()


MP = json.load(open(os.path.join(HERE, "golden", "multipaxos.json")))


@pytest.mark.parametrize("shards", [0, 3])
@pytest.mark.parametrize("name", sorted(MP))
def test_ir_multipaxos_matches_golden(name, shards):
    """BASELINE C5's protocol generated from the IR (dslabs_amd/ir/specs/multipaxos.py) on the
    MI355X engine: every multipaxos.json fixture of the hand-written protocol -- C5 to depth 12
    included -- per depth, also hash-sharded over 3 virtual shards (C5 d12 too); terminal traces replay on the
    IR-generated oracle form."""
    from test_ir import _mp_ir
    case = MP[name]
    proto, rest = _mp_ir(case["args"])
    e = Engine(proto, virtual_shards=shards, replicate_below=0 if shards else -1)
    try:
        r = e.bfs(proto.initial_state(), argmap.settings(rest, proto, table_log2=22))
    finally:
        e.close()
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"]
    st = r.invariantViolatingState() or r.goalMatchingState()
    if st is not None:
        rep = oracle_util.replay(proto.oracle_args() + [a for a in rest if a != "--finish-level"], st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth()


PBG = json.load(open(os.path.join(HERE, "golden", "pb.json")))


@pytest.mark.parametrize("shards", [0, 3])
@pytest.mark.parametrize("name", sorted(PBG))
def test_ir_pb_matches_golden(name, shards):
    """lab2 PB generated from the IR (dslabs_amd/ir/specs/pb.py: argument and network predicates)
    on the MI355X engine against every pb.json fixture, also hash-sharded over 3 virtual shards;
    terminal traces replay on the IR-generated oracle form."""
    from test_ir import _pb_ir, _pb_oracle_args
    case = PBG[name]
    proto, rest = _pb_ir(case["args"])
    e = Engine(proto, virtual_shards=shards, replicate_below=0 if shards else -1)
    try:
        r = e.bfs(proto.initial_state(), argmap.settings(rest, proto, table_log2=22))
    finally:
        e.close()
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"]
    st = r.invariantViolatingState() or r.goalMatchingState()
    if st is not None:
        rep = oracle_util.replay(_pb_oracle_args(proto, [a for a in rest if a != "--finish-level"]), st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth()


def _lab3():
    from test_gpu_multipaxos import LIVE
    return LIVE


@pytest.mark.parametrize("name", sorted(_lab3()))
def test_ir_multipaxos_lab3_predicates(name):
    """PaxosTest's argument predicates (slotValid, hasStatus, hasCommand, in combinators) on the
    IR-generated Multi-Paxos on the MI355X engine: the hand-written protocol's oracle run, per
    depth; terminal traces replay on the IR oracle."""
    from test_ir import _mp_ir, _mp_oracle_args
    args = _lab3()[name]
    want = oracle_util.run("bfs", args + ["--finish-level"], timeout=300)
    proto, rest = _mp_ir(args)
    r = Engine(proto).bfs(proto.initial_state(), argmap.settings(rest, proto, table_log2=20))
    assert r.endCondition().name == want["end"]
    assert r.per_depth == want["per_depth"]
    st = r.invariantViolatingState() or r.goalMatchingState()
    if st is not None:
        rep = oracle_util.replay(_mp_oracle_args(proto, rest), st.trace())
        assert rep["ok"], rep["error"]
        assert rep["depth"] == st.depth()
