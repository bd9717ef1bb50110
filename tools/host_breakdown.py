"""Host time of one C5 d12 step, split: SearchSettings preparation (Engine._prepare), the engine's
dsl_run (C++: setup, queued levels, waits, results) and the Python result objects (_results), over
N searches after a warm-up; the engine's own elapsed time is printed beside them.
usage: python tools/host_breakdown.py [N=40]"""
import ctypes
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dslabs_amd import Engine, _lib  # noqa: E402
from dslabs_amd._lib import check  # noqa: E402

proto, s, _ = bench.build_search("multipaxos", 12)
eng = Engine(proto, device=0)
st = proto.initial_state()
for _ in range(5):
    eng.bfs(st, s)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
prep, run, res, eng_el = [], [], [], []
for _ in range(n):
    t0 = time.perf_counter()
    eng._prepare(st, s)
    t1 = time.perf_counter()
    rp = ctypes.POINTER(_lib.dsl_result)()
    check(eng.lib.dsl_run(eng.handle, ctypes.byref(rp)), "dsl_run")
    t2 = time.perf_counter()
    r = eng._results(st, s, rp)
    t3 = time.perf_counter()
    prep.append(t1 - t0)
    run.append(t2 - t1)
    res.append(t3 - t2)
    eng_el.append(r.elapsed_s)
med = lambda x: 1e6 * statistics.median(x)  # noqa: E731
print(f'{{"prepare_us": {med(prep):.1f}, "dsl_run_us": {med(run):.1f}, "results_us": {med(res):.1f}, '
      f'"engine_elapsed_us": {med(eng_el):.1f}, "searches": {n}}}')
