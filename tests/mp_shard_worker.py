"""Worker for tests: one shard of a multi-process search (gloo host transport).

env: RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT; argv: <mode> <out.json>
mode 'collectives' runs the dsl_host_comm callbacks directly (CPU only);
mode 'lab0' / 'sipaxos' / 'mutant' / 'mp_c5' runs a sharded search on cuda:0 through the engine."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    mode, out = sys.argv[1], sys.argv[2]
    if mode == "dead_peer":  # a dead peer must surface as an error within seconds, not gloo's 30 min
        import datetime
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=20))
    else:
        dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from dslabs_amd.distributed import TorchHostComm
    # DSL_TEST_DEVICE_COLLECTIVES=1: the engine runs its RCCL branches (device-side gathers), the
    # gathers emulated over gloo (DSL_HOST_COMM_DEVICE_COLLECTIVES)
    hc = TorchHostComm(device_collectives=os.environ.get("DSL_TEST_DEVICE_COLLECTIVES") == "1")
    res = {"rank": rank}
    if mode == "collectives":
        U = ctypes.POINTER(ctypes.c_uint64)
        inp = np.array([rank + 1, 10 * (rank + 1)], dtype=np.uint64)
        outa = np.zeros(2 * world, dtype=np.uint64)
        hc.allgather(None, inp.ctypes.data_as(U), 2, outa.ctypes.data_as(U))
        res["allgather"] = outa.tolist()
        v = np.array([rank + 5, ~np.uint64(0) if rank == 0 else np.uint64(7)], dtype=np.uint64)
        hc.allreduce(None, v.ctypes.data_as(U), 2, 1)
        res["allreduce_min"] = [int(x) for x in v]
        v = np.array([rank + 5, 1 << 40], dtype=np.uint64)
        hc.allreduce(None, v.ctypes.data_as(U), 2, 0)
        res["allreduce_sum"] = [int(x) for x in v]
        b = np.array([rank * 3 + 1, rank], dtype=np.uint64)
        hc.bcast(None, b.ctypes.data_as(U), 2, world - 1)
        res["bcast"] = [int(x) for x in b]
        # alltoallv: rank r sends (r*16 + d) repeated (r + d + 1) times to rank d, region stride 64
        so = np.array([64 * d for d in range(world)], dtype=np.uint64)
        sb = np.array([0 if d == rank else rank + d + 1 for d in range(world)], dtype=np.uint64)
        send = np.zeros(64 * world, dtype=np.uint8)
        for d in range(world):
            send[64 * d: 64 * d + int(sb[d])] = rank * 16 + d
        rb = np.array([0 if s == rank else s + rank + 1 for s in range(world)], dtype=np.uint64)
        ro = np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.uint64)
        recv = np.zeros(int(rb.sum()) + 1, dtype=np.uint8)
        U8 = ctypes.POINTER(ctypes.c_uint8)
        hc.alltoallv(None, send.ctypes.data_as(U8), so.ctypes.data_as(U), sb.ctypes.data_as(U),
                     recv.ctypes.data_as(U8), ro.ctypes.data_as(U), rb.ctypes.data_as(U))
        res["alltoallv"] = recv[:int(rb.sum())].tolist()
    elif mode == "dead_peer":
        # both ranks search C5 to depth 8, every level sharded; then rank 1 dies; rank 0's next
        # search must fail with DSL_ERR_COMM and every later one be refused at once
        import time
        from dslabs_amd import RESULTS_OK, Engine, SearchSettings
        from dslabs_amd._lib import EngineError
        from dslabs_amd.protocols import MultiPaxos
        proto = MultiPaxos(3, 2, "append-xy")
        s = SearchSettings().addInvariant(RESULTS_OK).maxDepth(8)
        s.table_log2_slots = 22
        eng = Engine(proto, device=0, rank=rank, world_size=world, host_comm=hc, replicate_below=0)
        r = eng.bfs(proto.initial_state(), s)
        res["first"] = r.per_depth
        if rank == 1:
            with open(out, "w") as f:
                json.dump(res, f)
            os._exit(0)  # no goodbye to the peer
        time.sleep(1.0)
        for k in ("second", "third"):
            t0 = time.perf_counter()
            try:
                eng.bfs(proto.initial_state(), s)
                res[k] = "ok"
            except EngineError as e:
                res[k] = str(e)
            res[k + "_s"] = round(time.perf_counter() - t0, 3)
        with open(out, "w") as f:
            json.dump(res, f)
        os._exit(0)  # the process group cannot be torn down with the peer gone
    else:
        from dslabs_amd import CLIENTS_DONE, RESULTS_OK, Engine, SearchSettings
        from dslabs_amd.protocols import MultiPaxos, PingPong, SIPaxos
        if mode.startswith("synth_c3_d"):  # BASELINE C3 (bench.py's workload) to a smaller maxDepth
            sys.path.insert(0, ROOT)
            import bench
            proto, s, _ = bench.build_search("synthetic", int(mode[len("synth_c3_d"):]))
        elif mode == "mp_c5":  # BASELINE C5 at maxDepth 12 (levels above replicate_below are sharded)
            proto = MultiPaxos(3, 2, "append-xy")
            s = SearchSettings().addInvariant(RESULTS_OK).addInvariant(proto.predicate("LOGS_CONSISTENT_ALL_SLOTS"))
            s.addInvariant(proto.predicate("APPENDS_LINEARIZABLE")).maxDepth(12)
        elif mode == "lab0":
            proto = PingPong(2, 10)
            s = SearchSettings().addInvariant(RESULTS_OK).addPrune(CLIENTS_DONE)
        elif mode == "mutant":
            proto = PingPong(1, 10, check_value=False)
            s = SearchSettings().addInvariant(RESULTS_OK).addGoal(CLIENTS_DONE)
        else:
            proto = SIPaxos(2, 3, ("a", "b"))
            s = SearchSettings().addInvariant(proto.predicate("Integrity")).addInvariant(proto.predicate("Agreement"))
            s.maxDepth(9)
        s.table_log2_slots = 23 if mode in ("mp_c5",) or mode.startswith("synth") else 22
        rb = int(os.environ.get("DSL_TEST_REPLICATE_BELOW", "0"))
        eng = Engine(proto, device=0, rank=rank, world_size=world, host_comm=hc, replicate_below=rb)
        first = None
        if mode == "mp_c5" or mode.startswith("synth"):  # warm-up: buffers grow in the first search
            r0 = eng.bfs(proto.initial_state(), s)
            st0 = eng.kernel_stats()
            first = dict(per_depth=r0.per_depth, exchanged=st0["exchanged"], sharded_levels=st0["sharded_levels"],
                         shard_work_min=st0["shard_work_min"])
        r = eng.bfs(proto.initial_state(), s)
        st = eng.kernel_stats()
        res.update(end=r.endCondition().name, per_depth=r.per_depth, states=r.states, exchanged=st["exchanged"],
                   host_syncs=st["host_syncs"], sharded_levels=st["sharded_levels"], first=first,
                   fast_levels=st["fast_levels"], completions=st["completions"],
                   exchange_rounds=st["exchange_rounds"],
                   cost_c_ns=st["cost_c_ns"], cost_x_us=st["cost_x_us"], shard_work_min=st["shard_work_min"])
        t = r.invariantViolatingState() or r.goalMatchingState()
        if t is not None:
            res["trace"] = t.trace()
            res["depth"] = t.depth()
        eng.close()
    res["errors"] = hc.errors
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
