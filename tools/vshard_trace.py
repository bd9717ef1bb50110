"""C5 searches on virtual shards with DSL_LEVEL_TRACE (set by the caller): which buffers grow in
which search, and the cost model's state after each search.
usage: python tools/vshard_trace.py SHARDS REPLICATE_BELOW [SEARCHES] [DEPTH]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dslabs_amd import Engine  # noqa: E402

shards, rep = int(sys.argv[1]), int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 3
depth = int(sys.argv[4]) if len(sys.argv) > 4 else 12
proto, s, _ = bench.build_search("multipaxos", depth)
eng = Engine(proto, virtual_shards=shards, replicate_below=rep)
for i in range(n):
    print(f"=== search {i}", file=sys.stderr, flush=True)
    r = eng.bfs(proto.initial_state(), s)
    st = eng.kernel_stats()
    print(f"[stats] search {i}: {1e3 * r.elapsed_s:.3f} ms sharded={st['sharded_levels']} c={st['cost_c_ns']:.4f} "
          f"x={st['cost_x_us']:.1f} min={st['shard_work_min']} rehash={st['table_rehashes']}", file=sys.stderr, flush=True)
