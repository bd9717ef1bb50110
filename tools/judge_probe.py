"""Cost of each C5 invariant in k_level: the bench workload (Multi-Paxos 3 servers / 2 clients,
maxDepth 12) searched with every subset of its three invariants; kernel time per search (HIP
events, Engine.kernel_stats) over N repeats, after a warmup. Measurement tool (GPU box):
python3 tools/judge_probe.py [N]"""
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dslabs_amd import RESULTS_OK, Engine, SearchSettings  # noqa: E402
from dslabs_amd.protocols import MultiPaxos  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    proto = MultiPaxos(3, 2, "append-xy")
    preds = {"RESULTS_OK": RESULTS_OK, "LOGS": proto.predicate("LOGS_CONSISTENT_ALL_SLOTS"),
             "APPENDS": proto.predicate("APPENDS_LINEARIZABLE")}
    eng = Engine(proto)
    try:
        for k in range(len(preds) + 1):
            for names in itertools.combinations(preds, k):
                s = SearchSettings()
                for x in names:
                    s.addInvariant(preds[x])
                s.maxDepth(12)
                s.table_log2_slots = 22
                eng.bfs(proto.initial_state(), s)
                ms = []
                for _ in range(n):
                    eng.bfs(proto.initial_state(), s)
                    ms.append(eng.kernel_stats()["expand_ms"])
                ms.sort()
                print(json.dumps({"invariants": list(names), "expand_ms_median": round(ms[len(ms) // 2], 4),
                                  "expand_ms_min": round(ms[0], 4)}), flush=True)
    finally:
        eng.close()


if __name__ == "__main__":
    main()
