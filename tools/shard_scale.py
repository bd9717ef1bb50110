"""Sharded C3 (BASELINE configs[2], the dedup / all-to-all stress test) at scale on one GPU:
virtual shards run the multi-GPU engine's every phase (k_level<ROUTE>, slab exchange rounds as
device copies, owner probes, materialization, level records) one shard after another, so per-depth
counts, routing buffers and per-level exchange volume are exercised at 1e8 states; the timing
measures the emulation, not xGMI. usage: python3 tools/shard_scale.py [--workload multipaxos] DEPTH W [W ...]
> out.jsonl (per-level [level] / [shard] lines of DSL_LEVEL_TRACE go to stderr; the replicate_below
threshold from DSL_SCALE_REPLICATE_BELOW, default 100000)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from dslabs_amd import Engine  # noqa: E402


def main():
    args = sys.argv[1:]
    workload = "synthetic"
    if args[0] == "--workload":
        workload, args = args[1], args[2:]
    depth = int(args[0])
    rep = int(os.environ.get("DSL_SCALE_REPLICATE_BELOW", "100000"))
    gold = os.path.join(ROOT, "tests", "golden")
    if workload == "synthetic":
        want = json.load(open(os.path.join(gold, "deep.json")))["synth_c3_d10_cpu_bfs"]["per_depth"][:depth + 1]
    else:
        want = json.load(open(os.path.join(gold, "deep.json")))["mp_c5_d14"]["per_depth"][:depth + 1]
    proto, s, _ = bench.build_search(workload, depth)
    s.table_log2_slots = 26 if workload == "synthetic" else 23
    for w in [int(x) for x in args[1:]]:
        eng = Engine(proto, virtual_shards=w, replicate_below=rep) if w > 1 else Engine(proto)
        try:
            for run in range(2):  # the first search grows every buffer
                print(f"---- W={w} search {run}", file=sys.stderr, flush=True)
                t0 = time.perf_counter()
                r = eng.bfs(proto.initial_state(), s)
                el = time.perf_counter() - t0
                st = eng.kernel_stats()
                print(json.dumps({"workload": f"{workload} maxDepth {depth}", "virtual_shards": w,
                                  "replicate_below": rep, "search": run, "states": r.states,
                                  "per_depth_equal_cpu_bfs": r.per_depth == want, "elapsed_s": round(el, 4),
                                  "expand_ms": round(st["expand_ms"], 3), "exchange_ms": round(st["exchange_ms"], 3),
                                  "sharded_levels": st["sharded_levels"], "fast_levels": st["fast_levels"],
                                  "completions": st["completions"], "exchange_rounds": st["exchange_rounds"],
                                  "routed_records": st["exchanged"], "routed_bytes": st["exchanged"] * 12,
                                  "host_syncs": st["host_syncs"], "table_slots": st["table_slots"]}), flush=True)
                assert r.per_depth == want, (r.per_depth, want)
        finally:
            eng.close()


if __name__ == "__main__":
    main()
