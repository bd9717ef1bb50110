"""Deep searches against the oracle's deep fixtures (tests/golden/deep.json, generated on request by
make_golden.py deep: the oracle needs tens of minutes for each). BASELINE C5 to maxDepth 14
(8,808,218 states) from the default first table of 2^20 slots -- the visited table grows -- and
on virtual shards; IncorrectSingleInstancePaxos to its first Agreement violation at depth 14."""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import EndCondition, Engine

pytestmark = pytest.mark.gpu
DEEP = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "deep.json")))


def _run(case, table_log2=0, **eng):
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto, table_log2=table_log2)
    e = Engine(proto, **eng)
    try:
        return e.bfs(proto.initial_state(), s), e.kernel_stats()
    finally:
        e.close()


@pytest.mark.parametrize("log2,eng", [(20, {}), (0, {}), (20, {"virtual_shards": 4})])
def test_c5_depth14_grows_from_a_small_table(log2, eng):
    case = DEEP["mp_c5_d14"]
    r, st = _run(case, log2, **eng)
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"]
    assert r.states == case["states"] == 8808218
    assert st["table_rehashes"] >= 1


@pytest.mark.skipif("sipaxos_incorrect_d14" not in DEEP, reason="fixture not generated")
def test_incorrect_sipaxos_depth14():
    case = DEEP.get("sipaxos_incorrect_d14")
    r, _ = _run(case, 24)
    assert r.endCondition().name == case["end"] == "INVARIANT_VIOLATED"
    assert r.per_depth == case["per_depth"]
    st = r.invariantViolatingState()
    assert st.depth() == case["terminal_depth"] == 14
    rep = oracle_util.replay([a for a in case["args"] if a != "--finish-level"], st.trace())
    assert rep["ok"], rep["error"]
    assert rep["depth"] == 14 and not all(i["value"] for i in rep["invariants"])


@pytest.mark.parametrize("name", ["synth_c3_d7", "synth_c3_d8"])
def test_synthetic_c3_deep(name):
    """BASELINE C3 through depth 7 and 8 (30,341,487 states, the deepest oracle
    pin: 19 minutes on the oracle) against the oracle; the bench's depth 10 is checked through its
    prefix (tests/test_gpu_synthetic.py)."""
    if name not in DEEP:
        pytest.skip("fixture not generated")
    case = DEEP[name]
    r, _ = _run(case, 24 if name == "synth_c3_d7" else 27)
    assert r.endCondition().name == case["end"]
    assert r.per_depth == case["per_depth"]
    assert r.states == case["states"]
