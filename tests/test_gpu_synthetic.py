"""The table-driven synthetic protocol (BASELINE C3) on the MI355X engine vs the
oracle's golden vectors: per-depth counts, first-violation depth, replayable traces, sharding."""
import json
import os

import pytest

import argmap
import oracle_util
from dslabs_amd import EndCondition, Engine

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "synthetic.json")))


def _run(case, **eng):
    proto = argmap.protocol(case["args"])
    s = argmap.settings(case["args"], proto)
    e = Engine(proto, **eng)
    try:
        return e.bfs(proto.initial_state(), s)
    finally:
        e.close()


@pytest.mark.parametrize("name", sorted(GOLD))
def test_synthetic_parity(name):
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


@pytest.mark.parametrize("shards,rep", [(2, 0), (5, 0), (8, 0), (8, 1000)])
def test_synthetic_sharded(shards, rep):
    for name in ("synth_c3_d5", "synth_2n_k4_exhaustive"):
        case = GOLD[name]
        r = _run(case, virtual_shards=shards, replicate_below=rep)
        assert r.per_depth == case["per_depth"], (name, shards)


def test_synthetic_c3_bench_config_depth10(monkeypatch):
    """The C3 bench configuration itself (bench.py --workload synthetic: maxDepth 10, 780,909,037
    states, a 2^31-slot table far beyond the Infinity Cache), whole per-depth vector pinned
    independently of the kernels: equal to the multithreaded host BFS over the same transition
    functions run to the full depth in the build container (tests/golden/deep.json
    synth_c3_d10_cpu_bfs, `python tests/golden/make_golden.py deep-cpu`: a host visited set and host
    frontiers, not the device's), whose depth-0..8 prefix is the oracle's deepest pin (synth_c3_d8);
    both probe modes (load-first, the default at this table size; CAS-only) give that vector."""
    import sys
    deep = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "deep.json")))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    proto, s, _ = bench.build_search("synthetic", 10)
    e = Engine(proto)
    try:
        r = e.bfs(proto.initial_state(), s)
        monkeypatch.setenv("DSL_PROBE_LOAD", "0")
        r0 = e.bfs(proto.initial_state(), s)
    finally:
        e.close()
    cpu = deep["synth_c3_d10_cpu_bfs"]
    assert cpu["per_depth"][:9] == deep["synth_c3_d8"]["per_depth"]
    assert r.per_depth == r0.per_depth == cpu["per_depth"]
    assert r.states == cpu["states"] == 780909037


@pytest.mark.parametrize("shards", [2, 8])
def test_synthetic_c3_sharded_at_scale(shards):
    """BASELINE C3 (the dedup / all-to-all stress configuration) hash-sharded at 3e7 states:
    maxDepth 8 on virtual shards, levels past 100,000 frontier states sharded (slab exchange,
    owner probes, materialization; tools/shard_scale.py runs maxDepth 9). Per-depth counts equal
    the oracle's synth_c3_d8; the second search completes every sharded level on the fast path."""
    import sys
    deep = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "deep.json")))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    proto, s, _ = bench.build_search("synthetic", 8)
    s.table_log2_slots = 24
    e = Engine(proto, virtual_shards=shards, replicate_below=100000)
    try:
        r0 = e.bfs(proto.initial_state(), s)
        r = e.bfs(proto.initial_state(), s)
        st = e.kernel_stats()
    finally:
        e.close()
    assert r0.per_depth == r.per_depth == deep["synth_c3_d8"]["per_depth"]
    assert st["sharded_levels"] >= 2 and st["exchanged"] > 10 ** 6, st
    assert st["fast_levels"] == st["sharded_levels"] and st["completions"] == 0, st
