"""Multi-process (world_size 2+) sharding plumbing on CPU with gloo: the dsl_host_comm
collectives the sharded engine calls, and the RCCL id bootstrap."""
import json
import os
import socket
import subprocess
import sys
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_workers(mode, world, timeout=300, replicate_below=0, device_collectives=False, env=None):
    port = _free_port()
    outs, procs = [], []
    with tempfile.TemporaryDirectory() as d:
        for r in range(world):
            out = os.path.join(d, f"r{r}.json")
            outs.append(out)
            wenv = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                        MASTER_PORT=str(port), LOCAL_RANK="0", DSL_TEST_REPLICATE_BELOW=str(replicate_below),
                        DSL_TEST_DEVICE_COLLECTIVES="1" if device_collectives else "0")
            wenv.update(env or {})
            procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "mp_shard_worker.py"), mode, out],
                                          env=wenv))
        for p in procs:
            assert p.wait(timeout=timeout) == 0
        return [json.load(open(o)) for o in outs]


@pytest.mark.parametrize("world", [2, 3])
def test_host_comm_collectives_gloo(world):
    res = run_workers("collectives", world)
    for r in res:
        assert r["errors"] == []
        assert r["allgather"] == [x for k in range(world) for x in (k + 1, 10 * (k + 1))]
        assert r["allreduce_min"] == [5, 7]
        assert r["allreduce_sum"] == [sum(k + 5 for k in range(world)), world << 40]
        assert r["bcast"] == [(world - 1) * 3 + 1, world - 1]
        me = r["rank"]
        want = []
        for s in range(world):
            if s != me:
                want += [s * 16 + me] * (s + me + 1)
        assert r["alltoallv"] == want
