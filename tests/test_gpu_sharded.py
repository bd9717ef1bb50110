"""Sharded BFS on the GPU: per-depth counts are shard-count invariant and equal the oracle's."""
import json
import os

import pytest

from dslabs_amd import CLIENTS_DONE, RESULTS_OK, EndCondition, Engine, SearchSettings
from dslabs_amd.protocols import PingPong, SIPaxos
from test_distributed import run_workers

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LAB0 = json.load(open(os.path.join(GOLD, "lab0.json")))
SIP = json.load(open(os.path.join(GOLD, "sipaxos.json")))
MPX = json.load(open(os.path.join(GOLD, "multipaxos.json")))


@pytest.mark.parametrize("shards,rep", [(2, 0), (3, 0), (8, 0), (3, 40), (8, -1)])
def test_virtual_shards_lab0(shards, rep):
    """rep = replicate_below: 0 = hash-sharded from the first level, 40 = replicated small
    levels then sharded (crossover mid-search), -1 = default (this space stays replicated)."""
    eng = Engine(PingPong(2, 10), virtual_shards=shards, replicate_below=rep)
    s = SearchSettings().addInvariant(RESULTS_OK).addPrune(CLIENTS_DONE)
    s.table_log2_slots = 20
    r = eng.bfs(eng.protocol.initial_state(), s)
    assert r.endCondition() == EndCondition.SPACE_EXHAUSTED
    assert r.per_depth == LAB0["lab0_2c10p_exhaustive"]["per_depth"]
    assert (eng.kernel_stats()["exchanged"] > 0) == (rep >= 0)


@pytest.mark.parametrize("shards,rep", [(2, 0), (5, 0), (5, 100)])
def test_virtual_shards_sipaxos(shards, rep):
    proto = SIPaxos(2, 3, ("a", "b"))
    eng = Engine(proto, virtual_shards=shards, replicate_below=rep)
    s = SearchSettings().addInvariant(proto.predicate("Integrity")).addInvariant(proto.predicate("Agreement"))
    s.maxDepth(9)
    s.table_log2_slots = 22
    r = eng.bfs(proto.initial_state(), s)
    assert r.per_depth == SIP["sipaxos_2p3a_d9"]["per_depth"]


@pytest.mark.parametrize("shards,rep", [(2, 0), (4, 0), (4, -1)])
def test_virtual_shards_terminal_trace(shards, rep):
    eng = Engine(PingPong(1, 10, check_value=False), virtual_shards=shards, replicate_below=rep)
    s = SearchSettings().addInvariant(RESULTS_OK).addGoal(CLIENTS_DONE)
    s.table_log2_slots = 20
    r = eng.bfs(eng.protocol.initial_state(), s)
    assert r.endCondition() == EndCondition.INVARIANT_VIOLATED
    st = r.invariantViolatingState()
    assert st.depth() == 3
    assert st.trace() == LAB0["lab0_mutant_nocheck"]["pinned"]["trace"]


@pytest.mark.parametrize("mode,world,rep", [("lab0", 2, 0), ("sipaxos", 3, 0), ("mutant", 2, 0), ("lab0", 3, 40),
                                            ("sipaxos", 2, 100), ("mutant", 2, 40), ("mp_c5", 2, -1),
                                            ("mp_c5", 3, -1)])
def test_multiprocess_shards_one_gpu(mode, world, rep):
    """world processes on cuda:0, one shard each, exchanging through the gloo host transport;
    rep > 0: replicated small levels first (a terminal inside them walks a local chain)."""
    res = run_workers(mode, world, replicate_below=rep)
    for r in res:
        assert r["errors"] == []
    if mode == "lab0":
        want = LAB0["lab0_2c10p_exhaustive"]["per_depth"]
    elif mode == "sipaxos":
        want = SIP["sipaxos_2p3a_d9"]["per_depth"]
    elif mode == "mp_c5":  # the default replicate_below shards C5's largest levels
        want = MPX["mp_c5_d12"]["per_depth"]
    else:
        want = None
    for r in res:
        if want is not None:
            assert r["per_depth"] == want
        else:
            assert r["end"] == "INVARIANT_VIOLATED" and r["depth"] == 3
            assert r["trace"] == LAB0["lab0_mutant_nocheck"]["pinned"]["trace"]
    if mode == "mp_c5":  # automatic: the first search shards (default costs), every rank alike
        assert sum(r["first"]["exchanged"] for r in res) > 0
        assert len({(r["sharded_levels"], r["shard_work_min"]) for r in res}) == 1
    elif not (mode == "mutant" and rep > 0):
        assert sum(r["exchanged"] for r in res) > 0


@pytest.mark.parametrize("world", [2, 3])
def test_multiprocess_device_collectives_c5(world):
    """The RCCL engine's bookkeeping on gloo: with DSL_HOST_COMM_DEVICE_COLLECTIVES the engine takes
    its device-collective branches (the level records gathered on the device, bfs_engine.hpp
    gather_records), each gather emulated by the transport. C5 d12 with every level hash-sharded,
    then with the default threshold: per-depth counts equal the golden vector, states are routed,
    and (the second search, buffers grown) every sharded level is ONE host round trip on the slab
    fast path, the maxDepth level without round B."""
    want = MPX["mp_c5_d12"]["per_depth"]
    for rep in (0, -1):
        res = run_workers("mp_c5", world, replicate_below=rep, device_collectives=True)
        for r in res:
            assert r["errors"] == []
            assert r["per_depth"] == r["first"]["per_depth"] == want
            assert r["first"]["sharded_levels"] > 0
        assert sum(r["first"]["exchanged"] for r in res) > 0
        # every rank took the same decisions (the cost model is agreed in one collective)
        assert len({(r["sharded_levels"], r["shard_work_min"], r["fast_levels"]) for r in res}) == 1
        if rep == 0:
            for r in res:
                assert r["sharded_levels"] == 12
                assert r["fast_levels"] == 12 and r["completions"] == 0, r
                assert r["host_syncs"] <= r["sharded_levels"] + 1, r
                assert r["exchange_rounds"] == 2 * r["sharded_levels"] - 1, r  # no round B at maxDepth


@pytest.mark.parametrize("world,slab_max", [(2, 0), (3, 24)])
def test_multiprocess_sharded_completion_c5(world, slab_max):
    """The completion phase over gloo (device-collective branches): DSL_SLAB=0 sends every record
    through the host-sized rounds (round 4's two-round-trip exchange), DSL_SLAB_MAX=24 overflows
    every slab and region (records past the slab, route spills re-fingerprinted by k_respill):
    per-depth counts still equal the golden vector on every rank."""
    want = MPX["mp_c5_d12"]["per_depth"]
    env = {"DSL_SLAB": "0"} if slab_max == 0 else {"DSL_SLAB_MAX": str(slab_max)}
    res = run_workers("mp_c5", world, replicate_below=0, device_collectives=True, env=env)
    for r in res:
        assert r["errors"] == []
        assert r["per_depth"] == r["first"]["per_depth"] == want
        assert r["completions"] > 0, r


@pytest.mark.parametrize("rep", [0, -1])
def test_bench_multi_gpu_branch_share_device(rep):
    """bench.py's N > 1 branch end to end before the driver's 8-GPU run: torch.distributed.run
    starts 2 ranks of `bench.py --gpus 2` on the one GPU (DSL_BENCH_SHARE_DEVICE=1: gloo, the engine
    on the caller transport with its device-collective branches -- RCCL refuses two ranks on one
    device). Rank 0 prints the one JSON line: 2 GPUs, hash-sharded, per-depth counts equal C5 d12's
    golden vector, value = states x steps / the max-over-ranks time. rep 0: every level sharded,
    each on the one-round-trip fast path; rep -1: the cost model's choice (the driver's default)."""
    import subprocess
    import sys
    from test_distributed import _free_port
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DSL_BENCH_SHARE_DEVICE="1")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                        os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--replicate-below", str(rep)],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    b = json.loads(lines[0])
    assert b["n_gpus"] == 2 and b["steps"] == 3
    assert b["config"]["parallelism"] == "hash-sharded x2"
    assert b["config"]["per_depth"] == MPX["mp_c5_d12"]["per_depth"]
    assert "cpu_baseline" not in b
    sh = b["sharding"]
    want = b["config"]["unique_states_per_step"] * 3 / sh["elapsed_s_max_over_ranks"]
    assert abs(b["value"] - want) <= 1e-6 * want + 0.1  # value = round(., 1)
    assert sh["completions"] == 0
    if rep == 0:
        assert sh["sharded_levels"] == 12 and sh["fast_levels"] == 12, sh
        assert sh["exchanged_all_ranks"] > 0 and len(sh["per_rank"]) == 2
        assert sh["host_syncs"] <= sh["sharded_levels"] + 1, sh
        assert sh["exchange_rounds"] == 2 * sh["sharded_levels"] - 1, sh


def test_dead_peer_fails_the_search_and_refuses_later_ones():
    """a rank that dies between searches ends the survivor's next search with
    DSL_ERR_COMM (its transport's collective fails: here gloo's broken connection), and the engine
    refuses every later search at once instead of running out of step with its peers."""
    res = run_workers("dead_peer", 2, timeout=240)
    r0 = next(r for r in res if r["rank"] == 0)
    assert r0["first"] == MPX["mp_c5_d12"]["per_depth"][:9]
    assert "DSL_ERR_COMM" in r0["second"] and r0["second_s"] < 60, r0
    assert "DSL_ERR_COMM" in r0["third"] and "create a new engine" in r0["third"] and r0["third_s"] < 1, r0


def test_rccl_engine_at_world_1():
    """make_comm / ncclCommInitRank / ncclGetVersion and the RcclComm collectives run once on a
    one-GPU box: a world-size-1 engine with its RCCL communicator (DSL_CFG_RCCL_AT_WORLD_1) runs
    C5 to depth 8; the counts equal the golden prefix and the engine reports the RCCL it bound."""
    import argmap
    from dslabs_amd.distributed import comm_unique_id
    case = MPX["mp_c5_d12"]
    proto = argmap.protocol(case["args"])
    eng = Engine(proto, device=0, rank=0, world_size=1, comm_id=comm_unique_id(), rccl_at_world_1=True)
    try:
        s = argmap.settings(case["args"], proto, table_log2=20)
        s.maxDepth(8)
        r = eng.bfs(proto.initial_state(), s)
        st = eng.kernel_stats()
    finally:
        eng.close()
    assert r.per_depth == case["per_depth"][:9]
    assert st["rccl_version"] > 0, st


@pytest.mark.parametrize("shards", [2, 4, 8])
def test_virtual_shards_c5_default_settings(shards):
    """BASELINE C5 (d12) with the default replicate_below: the levels above it are hash-sharded
    (states routed), per-depth counts equal the golden vector."""
    import argmap
    case = MPX["mp_c5_d12"]
    proto = argmap.protocol(case["args"])
    eng = Engine(proto, virtual_shards=shards)
    try:
        r = eng.bfs(proto.initial_state(), argmap.settings(case["args"], proto, table_log2=23))
        st = eng.kernel_stats()
    finally:
        eng.close()
    assert r.per_depth == case["per_depth"]
    assert st["exchanged"] > 0 and st["sharded_levels"] > 0


@pytest.mark.parametrize("shards", [2, 8])
def test_sharded_level_host_round_trips(shards):
    """Every level hash-sharded (replicate_below = 0): on the slab fast path a sharded level is ONE
    host round trip (the gathered level records with the counters), the exchange rounds of virtual
    shards are one launch each (k_copy_segments), and the maxDepth level skips round B and
    k_materialize (its routed successors are judged at the source)."""
    import argmap
    case = MPX["mp_c5_d12"]
    proto = argmap.protocol(case["args"])
    eng = Engine(proto, virtual_shards=shards, replicate_below=0)
    try:
        s = argmap.settings(case["args"], proto, table_log2=23)
        eng.bfs(proto.initial_state(), s)  # warm-up: buffers grow in the first search
        r = eng.bfs(proto.initial_state(), s)
        st = eng.kernel_stats()
    finally:
        eng.close()
    assert r.per_depth == case["per_depth"]
    assert st["sharded_levels"] == 12
    assert st["fast_levels"] == 12 and st["completions"] == 0, st
    assert st["host_syncs"] <= st["sharded_levels"] + 1, st
    assert st["exchange_rounds"] == 2 * st["sharded_levels"] - 1, st


@pytest.mark.parametrize("shards,env", [(4, {"DSL_SLAB": "0"}), (4, {"DSL_SLAB_MAX": "16"}),
                                        (8, {"DSL_SLAB_MAX": "40"})])
def test_sharded_completion_phase(shards, env, monkeypatch):
    """Slabs too small for the level (DSL_SLAB_MAX) or none at all (DSL_SLAB=0): the records past
    each slab, the route-spilled successors (k_respill) and the spills past their room go through
    the completion phase; C5 d12 per-depth counts and a terminal trace stay exact."""
    import argmap
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    case = MPX["mp_c5_d12"]
    proto = argmap.protocol(case["args"])
    eng = Engine(proto, virtual_shards=shards, replicate_below=0)
    try:
        r = eng.bfs(proto.initial_state(), argmap.settings(case["args"], proto, table_log2=23))
        st = eng.kernel_stats()
    finally:
        eng.close()
    assert r.per_depth == case["per_depth"]
    assert st["completions"] > 0, st
    e2 = Engine(PingPong(1, 10, check_value=False), virtual_shards=shards, replicate_below=0)
    try:
        s = SearchSettings().addInvariant(RESULTS_OK).addGoal(CLIENTS_DONE)
        s.table_log2_slots = 20
        r2 = e2.bfs(e2.protocol.initial_state(), s)
    finally:
        e2.close()
    assert r2.endCondition() == EndCondition.INVARIANT_VIOLATED
    assert r2.invariantViolatingState().trace() == LAB0["lab0_mutant_nocheck"]["pinned"]["trace"]


def test_multiprocess_c3_gloo_device_collectives():
    """BASELINE C3 to maxDepth 7 (5.47 M states) over two processes (gloo, device-collective
    branches), the default cost rule: per-depth counts equal the oracle's synth_c3_d7 on both
    ranks, both ranks took identical sharding decisions."""
    deep = json.load(open(os.path.join(GOLD, "deep.json")))
    res = run_workers("synth_c3_d7", 2, replicate_below=-1, device_collectives=True)
    for r in res:
        assert r["errors"] == []
        assert r["per_depth"] == r["first"]["per_depth"] == deep["synth_c3_d7"]["per_depth"]
    assert len({(r["sharded_levels"], r["shard_work_min"], r["fast_levels"]) for r in res}) == 1
