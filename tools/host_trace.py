"""C5 d12 searches with DSL_LEVEL_TRACE (set by the caller): per-level host trace of the engine,
plus the Python-side time of each eng.bfs() call, for the host-overhead breakdown."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dslabs_amd import Engine  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 12
proto, s, _ = bench.build_search("multipaxos", depth)
eng = Engine(proto, device=0)
st = proto.initial_state()
for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
    t0 = time.perf_counter()
    r = eng.bfs(st, s)
    t1 = time.perf_counter()
    print(f"[py] search {i}: {1e3 * (t1 - t0):.4f} ms, engine elapsed {1e3 * r.elapsed_s:.4f} ms, states {r.states}",
          file=sys.stderr, flush=True)
