import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import json, argmap
from dslabs_amd import Engine
MPX = json.load(open("tests/golden/multipaxos.json"))
case = MPX["mp_c5_d12"]
proto = argmap.protocol(case["args"])
for W in (2, 3):
    eng = Engine(proto, virtual_shards=W, replicate_below=0)
    s = argmap.settings(case["args"], proto, table_log2=23)
    eng.bfs(proto.initial_state(), s)
    print("---- second search W", W, file=sys.stderr, flush=True)
    r = eng.bfs(proto.initial_state(), s)
    print(W, r.per_depth == case["per_depth"], eng.kernel_stats()["completions"], flush=True)
    eng.close()
