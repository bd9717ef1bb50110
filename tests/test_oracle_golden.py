"""The CPU oracle against the reference's own numbers (pinned) and the committed fixtures."""
import json
import os

import pytest

import oracle_util

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


LAB0 = _load("lab0.json")
SIP = _load("sipaxos.json")


@pytest.mark.parametrize("name", sorted(LAB0))
def test_lab0_oracle_matches_fixture_and_pins(name):
    case = LAB0[name]
    r = oracle_util.run("bfs", case["args"], timeout=300)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]
    assert r["states"] == case["states"] and r["max_depth"] == case["max_depth"]
    pin = case["pinned"]
    for k in ("states", "max_depth", "per_depth", "end"):
        if k in pin:
            assert {"states": r["states"], "max_depth": r["max_depth"], "per_depth": r["per_depth"],
                    "end": r["end"]}[k] == pin[k], (k, pin["source"])
    if "terminal_depth" in pin:
        assert r["terminals"][0]["depth"] == pin["terminal_depth"]
    if "trace" in pin:
        assert r["terminals"][0]["trace"] == pin["trace"]
    if "detail" in pin:
        assert r["terminals"][0]["detail"] == pin["detail"]


@pytest.mark.parametrize("name", ["sipaxos_2p3a_d6", "sipaxos_3p3a_d6", "sipaxos_2p3a_d9"])
def test_sipaxos_oracle(name):
    case = SIP[name]
    r = oracle_util.run("bfs", case["args"], timeout=300)
    assert r["per_depth"] == case["per_depth"]
    if "per_depth" in case["pinned"]:
        assert r["per_depth"] == case["pinned"]["per_depth"]


def test_timerqueue_truth_table():
    """TimerQueueTest.randomTimers: te1 always deliverable; te2 deliverable iff te2.min < te1.max."""
    tq = _load("timerqueue.json")
    r = oracle_util.run("timerqueue", [])
    assert r["cases"] == tq["cases"]
    assert len(r["cases"]) == 100
    for i, j, k, l, d1, d2l, d2i in r["cases"]:
        assert d1 == 1
        expect = 1 if k < j else 0
        assert d2l == expect and d2i == expect


def test_oracle_replay_readme_trace():
    """The README's mutant trace replays on the oracle and ends in the RESULTS_OK violation."""
    case = LAB0["lab0_mutant_nocheck"]
    args = [a for a in case["args"] if a != "--finish-level"]
    r = oracle_util.replay(args, case["pinned"]["trace"])
    assert r["ok"] and r["depth"] == 3
    assert r["invariants"][0]["value"] is False


SYN = _load("synthetic.json")


@pytest.mark.parametrize("name", sorted(SYN))
def test_synthetic_oracle_matches_fixture(name):
    case = SYN[name]
    r = oracle_util.run("bfs", case["args"], timeout=300)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


KVG = _load("amokv.json") if os.path.exists(os.path.join(GOLD, "amokv.json")) else {}


@pytest.mark.parametrize("name", sorted(n for n in KVG if n != "kv_3c_samekey3"))  # that one takes minutes
def test_amokv_oracle_matches_fixture(name):
    case = KVG[name]
    r = oracle_util.run("bfs", case["args"], timeout=300)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


PBG = _load("pb.json")


@pytest.mark.parametrize("name", sorted(PBG))
def test_pb_oracle_matches_fixture(name):
    case = PBG[name]
    r = oracle_util.run("bfs", case["args"], timeout=300)
    assert r["end"] == case["end"]
    assert r["per_depth"] == case["per_depth"]


def test_viewserver_passes_reference_unit_tests():
    """The oracle's ViewServer against the reference's own ViewServerTest scenarios (test01-12)."""
    r = oracle_util.run("vstest", [])
    names = [x["name"] for x in r["results"]]
    assert len(names) == 12 and names[0] == "test01StartupViewCorrect"
    assert all(x["ok"] for x in r["results"]), [x for x in r["results"] if not x["ok"]]


# SearchAndTraceMinimizerTest (framework/tst-self/dslabs/framework/testing/search/
# SearchAndTraceMinimizerTest.java): the reference's known answers for trace minimization.
MINI_TRACE = ["Message(a -> b, Foo())", "Message(a -> b, Foo())", "Message(b -> a, Bar())"]
MINI_TRACE2 = ["Message(a -> b, Foo())", "Message(a -> b, Foo())", "Message(b -> a, Foo())"]
MINI_CASES = [  # (name, settings args, trace, end, depth minimized, depth not minimized)
    ("testSearchMinimizesInvariantViolation", ["--inv", "foo"], MINI_TRACE, "INVARIANT_VIOLATED", 2, 3),
    ("testSearchMinimizesExceptionThrown", ["--inv", "foo"], MINI_TRACE2, "EXCEPTION_THROWN", 2, 3),
    ("testSearchMinimizesExceptionalPredicate", ["--inv", "fooException"], MINI_TRACE, "INVARIANT_VIOLATED", 2, 3),
    ("goalMinimization", ["--goal", "!foo"], MINI_TRACE, "GOAL_FOUND", 2, 3),
    ("exceptionsInGoal", ["--goal", "alwaysException"], MINI_TRACE, "SPACE_EXHAUSTED", 3, 3),
]


@pytest.mark.parametrize("case", MINI_CASES, ids=[c[0] for c in MINI_CASES])
def test_oracle_minimizer_reference_cases(case):
    _, sargs, trace, end, dmin, draw = case
    args = ["--proto", "minitest"] + sargs
    for minimize, depth in ((True, dmin), (False, draw)):
        r = oracle_util.replay_search(args, trace, minimize)
        assert r["end"] == end
        assert r["depth"] == depth
        assert len(r["trace"]) == depth


def test_oracle_human_readable_trace_drops_noop_steps():
    """SearchState.humanReadableTrace: the repeated Foo delivery changes nothing and is dropped;
    the causal order (b's Bar after a's Foo reached b) is kept."""
    r = oracle_util.replay_search(["--proto", "minitest", "--inv", "foo", "--human-readable"], MINI_TRACE, False)
    assert r["trace"] == ["Message(a -> b, Foo())", "Message(b -> a, Bar())"]
    assert r["depth"] == 2
