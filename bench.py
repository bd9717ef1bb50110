"""bench.py -- unique states explored / sec of the MI355X BFS engine (BASELINE.json metric).

A "step" is one complete BFS over the workload (Search.bfs from the initial state to the end
condition), timed with the search resident on the GPU; value = unique states (reference
counting rule, Search.java:470-490) x steps / wall time, whole job.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME] [--depth D]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

Multi-GPU: one process per GPU; the visited set and frontier are hash-partitioned by
fingerprint, successors routed to their owner shard per level (RCCL all-to-all over xGMI).
Per-depth counts are shard-count invariant; `value` = global unique states / max-rank time.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "unique states explored/sec (whole node) for Paxos BFS at 1/2/4/8 MI355X"  # BASELINE.json (C5)


def metric_name(workload: str) -> str:
    """BASELINE.json's metric names Paxos (C5, the default workload); another workload's line says
    which search it measured instead of passing for a Paxos number."""
    if workload in ("multipaxos", "multipaxos_ir"):
        return METRIC
    return f"unique states explored/sec (whole node) for {workload} BFS at 1/2/4/8 MI355X"
CPU_SAMPLE_S = 10.0  # seconds of timed CPU-baseline searches (a bounded sample)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
LLC_BYTES = 256 << 20  # MI355X Infinity Cache (MALL)

WORKLOADS = {
    # BASELINE config C5: lab3 Multi-Paxos (builder-authored), 3 servers, 2 clients
    # appending X / Y to one key, invariants RESULTS_OK + LOGS_CONSISTENT_ALL_SLOTS +
    # APPENDS_LINEARIZABLE, timers on, BFS to maxDepth 12 (1,110,019 unique states).
    "multipaxos": dict(depth=12, cpu_depth=10,
                       desc="lab3 Multi-Paxos, 3 servers + 2 clients (append X / append Y), invariants "
                            "RESULTS_OK, LOGS_CONSISTENT_ALL_SLOTS, APPENDS_LINEARIZABLE, timers on, BFS to maxDepth"),
    # The same C5 search on the protocol generated from the IR (dslabs_amd/ir/specs/multipaxos.py).
    "multipaxos_ir": dict(depth=12, cpu_depth=10,
                          desc="C5 on the IR-generated lab3 Multi-Paxos (dslabs_amd/ir/specs/multipaxos.py), "
                               "3 servers + 2 clients, the same invariants, BFS to maxDepth"),
    # The reference's own Paxos ("Paxos Made Simple", SingleInstancePaxos.java:50-127): 2
    # proposers, 3 acceptors, invariants Integrity + Agreement, exhaustive to maxDepth.
    # BASELINE config C3: the table-driven synthetic protocol, 5 nodes, 64-byte
    # packed state, ~20-25 successors per state, maxDepth 10 (~8e8 unique states).
    "synthetic": dict(depth=10, cpu_depth=6, cpu_mt_depth=8, table_log2=31,
                      desc="table-driven synthetic protocol (5 nodes, K=64, pokes at v%7==0, seed 0x5EEDD51AB5), "
                           "invariant NOT_ALL_MAX, BFS to maxDepth"),
    # BASELINE config C2: lab1 AMO KV, ClientServerPart2Test.test10 workload
    # (APPEND:foo:%i x 3, APPENDS_LINEARIZABLE, prune CLIENTS_DONE), exhaustive; "amokv3" = the
    # same with 3 clients (1,225,876 states).
    "amokv": dict(depth=-1, cpu_depth=-1, clients=2,
                  desc="lab1 AMO KV, 2 clients APPEND:foo:%i x3, APPENDS_LINEARIZABLE, prune CLIENTS_DONE, exhaustive"),
    "amokv3": dict(depth=-1, cpu_depth=14, clients=3,
                   desc="lab1 AMO KV, 3 clients APPEND:foo:%i x3, APPENDS_LINEARIZABLE, prune CLIENTS_DONE, exhaustive"),
    # BASELINE config C4: lab2 primary-backup + ViewServer, 2 servers, 1 client
    # putGetWorkload, RESULTS_OK, prunes CLIENTS_DONE and hasViewReply(INITIAL_VIEWNUM + 3).
    "pb": dict(depth=-1, cpu_depth=-1,
               desc="lab2 primary-backup + ViewServer, 2 servers, 1 client putGet, RESULTS_OK, prunes CLIENTS_DONE "
                    "and hasViewReply(4), exhaustive BFS from PrimaryBackupTest.initView(2, server1, server2) "
                    "(70,020 states, depth 42)"),
    "sipaxos": dict(depth=15, cpu_depth=10,
                    desc="reference SingleInstancePaxos (2 proposers, 3 acceptors), invariants "
                         "Integrity+Agreement, BFS to maxDepth"),
}


def build_search(name: str, depth: int):
    from dslabs_amd import SearchSettings
    from dslabs_amd import RESULTS_OK
    from dslabs_amd import CLIENTS_DONE
    from dslabs_amd.protocols import PB, AmoKV, MultiPaxos, MultiPaxosIR, SIPaxos, Synthetic
    if name in ("multipaxos", "multipaxos_ir"):
        proto = (MultiPaxos if name == "multipaxos" else MultiPaxosIR)(3, 2, "append-xy")
        s = SearchSettings().addInvariant(RESULTS_OK).addInvariant(proto.predicate("LOGS_CONSISTENT_ALL_SLOTS"))
        s.addInvariant(proto.predicate("APPENDS_LINEARIZABLE"))
        s.maxDepth(depth)
        # first visited table: what the growth rule (BfsEngine::ensure_table, at most half full
        # for the states inserted plus twice the estimate of the next level's) reaches at this
        # depth, so a timed search never rehashes; clearing it is part of every timed search
        s.table_log2_slots = max(20, min(32, 22 + (3 * (depth - 12) + 1) // 2))
        head = ["--proto", "multipaxos", "--workload", "append-xy"] if name == "multipaxos" else proto.oracle_args()
        return proto, s, head + ["--inv", "RESULTS_OK", "--inv", "LOGS_CONSISTENT_ALL_SLOTS", "--inv",
                                 "APPENDS_LINEARIZABLE"]
    if name == "pb":
        proto = PB(2, 1, "putget")
        s = SearchSettings().addInvariant(RESULTS_OK).addPrune(CLIENTS_DONE).addPrune(proto.predicate("hasViewReply:4"))
        s.maxDepth(depth)
        s.table_log2_slots = 28
        return proto, s, ["--proto", "pb", "--servers", "2", "--clients", "1", "--workload", "putget", "--inv",
                          "RESULTS_OK", "--prune", "CLIENTS_DONE", "--prune", "hasViewReply:4"]
    if name in ("amokv", "amokv3"):
        c = WORKLOADS[name]["clients"]
        proto = AmoKV(c, "samekey3")
        s = SearchSettings().addInvariant(proto.predicate("APPENDS_LINEARIZABLE")).addPrune(CLIENTS_DONE)
        s.maxDepth(depth)
        s.table_log2_slots = 24
        return proto, s, ["--proto", "amokv", "--clients", str(c), "--workload", "samekey3", "--inv",
                          "APPENDS_LINEARIZABLE", "--prune", "CLIENTS_DONE"]
    if name == "synthetic":
        proto = Synthetic(5, 64, 7)
        s = SearchSettings().addInvariant(proto.predicate("NOT_ALL_MAX"))
        s.maxDepth(depth)
        s.table_log2_slots = WORKLOADS[name].get("table_log2", 28) if depth >= 10 else 28
        return proto, s, ["--proto", "synthetic", "--inv", "NOT_ALL_MAX"]
    if name == "sipaxos":
        proto = SIPaxos(2, 3, ("a", "b"))
        s = SearchSettings().addInvariant(proto.predicate("Integrity")).addInvariant(proto.predicate("Agreement"))
        s.maxDepth(depth)
        s.table_log2_slots = 28
        return proto, s, ["--proto", "sipaxos", "--proposers", "2", "--acceptors", "3", "--values", "a,b",
                          "--inv", "Integrity", "--inv", "Agreement"]
    raise SystemExit(f"unknown workload {name}")


def cpu_baseline(proto, settings, depth: int, gpu_per_depth, oracle_args, oracle_depth: int, state=None) -> dict:
    """SURVEY.md §8(d)'s CPU baseline: the multithreaded level-synchronous BFS of
    tools/cpu_bfs.cpp (the reference's BFS worker scheme, Search.java:241-348, over the same packed
    transition functions, a lock-free visited set and a barrier per level) on this host's cores,
    on the SAME workload and maxDepth as the GPU line; a warm-up search (it grows the buffers,
    as the GPU's warmup step does), then repeated searches for a bounded ~10 s sample. `oracle_sample` is the scalar
    string-keyed oracle (oracle/, the reference's object model restated) on a smaller maxDepth: a
    reference-semantics sample, not the baseline."""
    sys.path.insert(0, ROOT)
    from tools import cpu_baseline as cb
    s = settings.clone()
    s.maxDepth(depth)
    r = cb.run(proto, s, repeat=2, min_seconds=CPU_SAMPLE_S, state=state if state is not None and state.packed else None)
    out = {"value": round(r["states_per_s"], 1), "unit": "states/s", "cores": r["threads"],
           "kind": "cpu_ref multithreaded",
           "sample": f"same workload, maxDepth {depth}: {r['runs']} searches of {r['states']} states in "
                     f"{r['timed_s']:.2f} s on {r['threads']} threads (tools/cpu_bfs.cpp)",
           "per_depth_equal_gpu": r["per_depth"] == gpu_per_depth[:len(r["per_depth"])]}
    if oracle_depth > 0:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        exe = os.path.join(ROOT, "oracle", "_build", "dslabs_oracle")
        o = subprocess.run([exe, "bfs"] + oracle_args + ["--max-depth", str(oracle_depth)], check=True,
                           capture_output=True, text=True, timeout=300)
        ro = json.loads(o.stdout)
        out["oracle_sample"] = {"value": round(ro["states"] / ro["elapsed_s"], 1), "cores": 1,
                                "sample": f"oracle/dslabs_oracle (scalar, string-keyed object model), maxDepth "
                                          f"{oracle_depth}, {ro['states']} states, {ro['elapsed_s']:.2f} s"}
    return out


def pmc_profile(workload: str, depth: int):
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}_d{depth}.json")))
    return json.load(open(fs[-1])) if fs else None


def pmc_traffic(workload: str, depth: int, launches: int, staged_bytes: int = 0):
    """HBM bytes per k_level launch from the committed rocprofv3 PMC summary of the same
    workload (tools/gpu_prof.sh + tools/pmc_summary.py, separate --pmc passes over one search),
    divided by this run's launches per search; None if this workload has no summary.
    Calibrated on gfx950 with tools/hbm_calib.hip (profiles/r01_hbm_calibration.json):
    FETCH_SIZE counts the random 64-B bucket-line reads exactly but only half of the 16-B/lane
    streaming reads, i.e. the staging of the frontier rows and fingerprints (`staged_bytes` per
    search), so traffic = FETCH_SIZE + staged_bytes / 2 + WRITE_SIZE."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}_d{depth}.json"))):
        best = f
    if best is None:
        return None, None
    d = json.load(open(best))
    if d.get("fetch_bytes_per_step") is not None and d.get("write_bytes_per_step") is not None:
        t = d["fetch_bytes_per_step"] + staged_bytes / 2 + d["write_bytes_per_step"]
        return int(t / max(1, launches)), os.path.relpath(best, ROOT)
    if d.get("hbm_bytes_per_step"):
        return int(d["hbm_bytes_per_step"] / max(1, launches)), os.path.relpath(best, ROOT)
    v = d.get("hbm_bytes_per_launch")
    return (int(v) if v else None), os.path.relpath(best, ROOT)


def roofline(stats: dict, workload: str, depth: int) -> dict:
    """Algorithmic bytes of k_level per launch, SURVEY.md §8(d)'s per-unique-state figure
    B_state = b·64 + 2·S + 72 summed exactly over the level: every generated successor costs one
    64-byte random visited-table line (the reference's discovered.add per successor,
    Search.java:485), every expanded parent is read once and every appended state written once (S
    bytes + its 16-byte fingerprint here), and every newly discovered state writes back its bucket
    line plus 8 bytes of parent / event (72); divided by the summed k_level durations (HIP events on
    the engine's stream). `achieved_probe_model` is the stricter count this engine can claim for
    itself: 64 bytes only per successor it actually probes (a successor that changes nothing is its
    parent and is never looked up)."""
    S = stats["state_bytes"]
    alg = (stats["parents"] * (S + 16) + stats["work_items"] * 64 + stats["new_states"] * 72
           + stats["appended"] * (S + 16))
    alg_probe = stats["parents"] * (S + 16) + stats["probes"] * 64 + stats["appended"] * (S + 16 + 12)
    t = stats["expand_ms"] / 1e3
    achieved = alg / t / 1e9 if t > 0 else 0.0
    achieved_probe = alg_probe / t / 1e9 if t > 0 else 0.0
    launches = max(1, stats["expand_launches"])
    traffic, src = pmc_traffic(workload, depth, launches, stats["parents"] * (S + 16))
    out = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
           "kernel": "k_level", "launches": stats["expand_launches"],
           "avg_launch_ms": round(stats["expand_ms"] / launches, 4),
           "alg_bytes_per_launch": int(alg / launches), "byte_model": "SURVEY.md 8(d): b*64 + 2*S + 72 per state",
           "achieved_probe_model": round(achieved_probe, 2), "frac_probe_model": round(achieved_probe / HBM_PEAK_GBS, 4)}
    if src:
        out["traffic_source"] = src
    # visited-set atomics (north_star): one 64-bit CAS per inserted state (live, HIP events), the
    # probes (bucket lookups) behind them, the table's size, and the PMC count of every atomic at
    # the L2 (TCC_ATOMIC, the committed profile of the same workload) per search
    out["level_slots"] = stats["level_slots"]  # k_level workgroups resident at once (the grid)
    out["atomics_per_s"] = round(stats["new_states"] / t, 1) if t > 0 else 0.0
    out["probes_per_s"] = round(stats["probes"] / t, 1) if t > 0 else 0.0
    # where the visited table lives: a table within the 256 MiB Infinity Cache (MALL) keeps the
    # probes' lines on chip, so that regime is bound by latency, not by HBM bandwidth (the 8 TB/s
    # denominator above then states how far the kernel is from the HBM roofline, not its bound)
    out["table_bytes"] = int(stats["table_slots"] * 8)
    out["llc_bytes"] = LLC_BYTES
    out["llc_resident"] = out["table_bytes"] <= LLC_BYTES
    out["regime"] = "latency (table in the Infinity Cache)" if out["llc_resident"] else "hbm random access"
    prof = pmc_profile(workload, depth)
    if prof and prof.get("atomics_per_step") is not None:
        out["pmc_atomics_per_search"] = int(prof["atomics_per_step"])
    ra = random_access_roofline(out["table_bytes"], out["probes_per_s"], out["atomics_per_s"])
    if ra:
        out["random_access"] = ra
    return out


def random_access_roofline(table_bytes: int, probes_per_s: float, inserts_per_s: float):
    """The probes' own ceiling: the chip-wide rates of independent random 64-B line loads and of
    random 8-byte agent-scope CAS on a table of about this size (tools/rand_calib.hip, committed
    as profiles/r04_random_access_calibration.jsonl; 16 waves per CU, 8 in flight per lane).
    A table beyond 1 GiB is probed by a load and only a new state's slot is CAS'd (fingerprint.hpp
    load_first), a smaller one by a CAS per probe. `time_share` = the fraction of the kernel's time
    those accesses alone would take at their ceilings (1.0 = at the random-access roofline)."""
    f = os.path.join(ROOT, "profiles", "r04_random_access_calibration.jsonl")
    if not os.path.exists(f):
        return None
    rows = [json.loads(x) for x in open(f) if x.strip()]
    rows = [r for r in rows if r.get("waves_per_cu") == 16] or rows
    import math
    r = min(rows, key=lambda r: abs(math.log2(r["table_bytes"]) - math.log2(max(1, table_bytes))))
    lc, cc = r["random_line_loads_per_s"], r["random_cas_per_s"]
    load_first = table_bytes > (1 << 30)
    share = (probes_per_s / lc + inserts_per_s / cc) if load_first else probes_per_s / cc
    return {"load_ceiling_per_s": lc, "cas_ceiling_per_s": cc, "calibrated_table_bytes": r["table_bytes"],
            "probe_mode": "load, then CAS if empty" if load_first else "CAS", "time_share": round(share, 4),
            "source": os.path.relpath(f, ROOT)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="multipaxos")
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # N > 1: the engine's replicated-or-sharded rule (Engine replicate_below): -1 = the cost model
    # (default), 0 = every level hash-sharded (tests), n > 0 = shard frontiers of at least n states
    ap.add_argument("--replicate-below", type=int, default=-1)
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # DSL_BENCH_SHARE_DEVICE=1 (rehearsal on a one-GPU box, never a bench line): every rank on
    # device 0 over gloo. RCCL refuses two ranks on one device, so the engine's transport is the
    # caller's (TorchHostComm) with DSL_HOST_COMM_DEVICE_COLLECTIVES: the engine takes the same
    # device-collective branches as with its RCCL communicator (level records gathered on the
    # device), each gather emulated by a device->host copy, the gloo allgather and a copy back
    share = os.environ.get("DSL_BENCH_SHARE_DEVICE") == "1"
    device = 0 if share else local_rank
    torch.cuda.set_device(device)
    dist = None
    comm_id = None
    host_comm = None
    if world > 1:
        import torch.distributed as dist
        if share:
            dist.init_process_group("gloo")
            from dslabs_amd.distributed import TorchHostComm
            host_comm = TorchHostComm(device_collectives=True)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            from dslabs_amd.distributed import broadcast_comm_id
            comm_id = broadcast_comm_id(rank)

    from dslabs_amd import Engine
    wl = WORKLOADS[args.workload]
    depth = args.depth if args.depth is not None else wl["depth"]
    proto, settings, oracle_args = build_search(args.workload, depth)
    eng = Engine(proto, device=device, rank=rank, world_size=world, comm_id=comm_id, host_comm=host_comm,
                 replicate_below=args.replicate_below)
    # C4 starts from PrimaryBackupTest.initView's prepared state (PrimaryBackupTest.java:124-187)
    state = proto.initView(2, "server1", "server2", "client1", device=device) if args.workload == "pb" \
        else proto.initial_state()

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.bfs(state, settings)
    barrier()
    t0 = time.perf_counter()
    total_states = 0
    res = None
    for _ in range(args.steps):
        res = eng.bfs(state, settings)
        total_states += res.states
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if share else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stats = eng.kernel_stats()
    per_rank = None
    if dist is not None:  # every rank's share of the last search (load balance of the shards)
        mine = {k: stats[k] for k in ("parents", "work_items", "new_states", "exchanged", "probes")}
        mine["expand_ms"] = round(stats["expand_ms"], 4)
        mine["exchange_ms"] = round(stats["exchange_ms"], 4)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    if rank == 0:
        line = {
            "metric": metric_name(args.workload),
            "workload": args.workload,
            "value": round(total_states / elapsed, 1),
            "unit": "states/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (model-checking state space generated from the protocol's initial state)",
            "config": {"workload": args.workload, "description": wl["desc"], "max_depth": depth,
                       "unique_states_per_step": res.states, "per_depth": res.per_depth,
                       "end_condition": res.endCondition().name, "state_bytes": stats["state_bytes"],
                       "successors_per_step": res.successors, "parallelism": f"hash-sharded x{world}"},
            "roofline": roofline(stats, args.workload, depth),
        }
        if world > 1:  # the last search's sharding bookkeeping (dsl_stats), rank 0's view
            line["sharding"] = {
                "transport": "gloo host comm, device-collective branches (one-GPU rehearsal)" if share
                else f"RCCL {stats['rccl_version']}",
                "elapsed_s_max_over_ranks": elapsed,
                **{k: stats[k] for k in ("sharded_levels", "fast_levels", "completions", "host_syncs",
                                         "exchange_rounds", "exchanged", "shard_work_min")},
                "cost_c_ns": round(stats["cost_c_ns"], 4), "cost_x_us": round(stats["cost_x_us"], 2),
                "exchanged_all_ranks": sum(r["exchanged"] for r in per_rank), "per_rank": per_rank}
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(proto, settings, min(depth, wl.get("cpu_mt_depth", depth)) if depth >= 0
                                                else depth, res.per_depth, oracle_args, wl["cpu_depth"], state)
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
