"""Per-level cost of the hash-sharded path on one GPU (virtual shards: exchanges are device
copies, so this shows the route/probe/materialize kernels and host syncs, not xGMI latency).
usage: DSL_LEVEL_TRACE=1 python tools/shard_probe.py SHARDS REPLICATE_BELOW [DEPTH]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dslabs_amd import Engine  # noqa: E402

shards, rep = int(sys.argv[1]), int(sys.argv[2])
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 12
proto, s, _ = bench.build_search("multipaxos", depth)
e = Engine(proto, virtual_shards=shards, replicate_below=rep)
for i in range(4):
    t = time.perf_counter()
    r = e.bfs(proto.initial_state(), s)
    dt = time.perf_counter() - t
    print(f"shards={shards} rep={rep} run {i}: {r.states} states {dt * 1e3:.3f} ms", file=sys.stderr, flush=True)
e.close()
