"""Per-level cost of the hash-sharded path on one GPU (virtual shards: the exchanges are device
copies, so this measures the route / probe / materialize kernels and the host synchronizations of
a sharded level, not xGMI latency). Prints one JSON line per configuration: ms per search, sharded
levels, exchanged records, and the added time per sharded level against the one-shard search.
usage: python tools/shard_probe.py [DEPTH] > out.jsonl"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dslabs_amd import Engine  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 12
proto, s, _ = bench.build_search("multipaxos", depth)


def measure(shards, rep, runs=5):
    e = Engine(proto, virtual_shards=shards, replicate_below=rep)
    try:
        e.bfs(proto.initial_state(), s)  # warmup: buffers
        best = None
        for _ in range(runs):
            t = time.perf_counter()
            r = e.bfs(proto.initial_state(), s)
            dt = time.perf_counter() - t
            st = e.kernel_stats()
            if best is None or dt < best[0]:
                best = (dt, r, st)
        return best
    finally:
        e.close()


base_dt, base_r, _ = measure(0, -1)
print(json.dumps({"shards": 1, "ms": round(base_dt * 1e3, 3), "states": base_r.states}), flush=True)
for shards in (2, 4, 8):
    for rep in (-1, 0, 16384):
        dt, r, st = measure(shards, rep)
        assert r.per_depth == base_r.per_depth
        lv = st["sharded_levels"]
        print(json.dumps({"shards": shards, "replicate_below": rep, "ms": round(dt * 1e3, 3),
                          "sharded_levels": lv, "exchanged": st["exchanged"],
                          "exchange_ms": round(st["exchange_ms"], 3), "cost_c_ns": round(st["cost_c_ns"], 2),
                          "cost_x_us": round(st["cost_x_us"], 1), "shard_work_min": st["shard_work_min"],
                          "added_ms_per_sharded_level": round((dt - base_dt) * 1e3 / lv, 4) if lv else None}),
              flush=True)
