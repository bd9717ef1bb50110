"""Multi-process sharded search plumbing.

* ``comm_unique_id`` / ``broadcast_comm_id``: rank 0 creates the RCCL id, torch.distributed carries
  it to the other ranks; the engine then builds its own RCCL communicator (one rank per GPU).
* ``TorchHostComm``: a ``dsl_host_comm`` (include/dslabs_hip.h) implemented with torch.distributed
  on CPU tensors (gloo). The engine uses it instead of RCCL when given one -- this is how the
  multi-process sharding protocol is exercised with several processes on ONE GPU (RCCL refuses
  two ranks per device) and how its collectives are unit-tested on CPU.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import numpy as np

from . import _lib

_U64P = ctypes.POINTER(ctypes.c_uint64)
_U8P = ctypes.POINTER(ctypes.c_uint8)
ALLGATHER = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _U64P, ctypes.c_int32, _U64P)
ALLREDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _U64P, ctypes.c_int32, ctypes.c_int32)
BCAST = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _U64P, ctypes.c_int32, ctypes.c_int32)
ALLTOALLV = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _U8P, _U64P, _U64P, _U8P, _U64P, _U64P)


class dsl_host_comm(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("rank", ctypes.c_int32), ("size", ctypes.c_int32),
                ("allgather_u64", ALLGATHER), ("allreduce_u64", ALLREDUCE), ("bcast_u64", BCAST),
                ("alltoallv", ALLTOALLV), ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_SIGN = np.uint64(1 << 63)


def _u64(ptr, n) -> np.ndarray:
    return np.ctypeslib.as_array(ptr, shape=(n,)) if n else np.zeros(0, np.uint64)


class TorchHostComm:
    """dsl_host_comm over a torch.distributed process group (CPU tensors, e.g. gloo)."""

    def __init__(self, group=None, device_collectives: bool = False):
        """device_collectives: DSL_HOST_COMM_DEVICE_COLLECTIVES -- the engine takes its RCCL code
        path (device-side gathers), each gather emulated through allgather (tests)."""
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.errors = []
        self._cbs = (ALLGATHER(self._wrap(self.allgather)), ALLREDUCE(self._wrap(self.allreduce)),
                     BCAST(self._wrap(self.bcast)), ALLTOALLV(self._wrap(self.alltoallv)))
        self.struct = dsl_host_comm(None, self.rank, self.size, *self._cbs,
                                    _lib.DSL_HOST_COMM_DEVICE_COLLECTIVES if device_collectives else 0, 0)

    def _wrap(self, fn):
        def cb(*args):
            try:
                fn(*args)
                return 0
            except Exception as e:  # noqa: BLE001 -- reported to the engine as DSL_ERR_COMM
                self.errors.append(repr(e))
                return 1
        return cb

    # --- collectives (also callable directly with numpy arrays, for tests) ----------------------
    def allgather(self, _ctx, inp, n, out):
        import torch
        x = torch.from_numpy(_u64(inp, n).view(np.int64).copy())
        parts = [torch.empty_like(x) for _ in range(self.size)]
        self.dist.all_gather(parts, x, group=self.group)
        _u64(out, n * self.size)[:] = torch.cat(parts).numpy().view(np.uint64)

    def allreduce(self, _ctx, v, n, is_min):
        import torch
        a = _u64(v, n)
        if is_min:  # order-preserving uint64 -> int64 map
            t = torch.from_numpy((a ^ _SIGN).view(np.int64).copy())
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
            a[:] = t.numpy().view(np.uint64) ^ _SIGN
        else:
            t = torch.from_numpy(a.view(np.int64).copy())
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
            a[:] = t.numpy().view(np.uint64)

    def bcast(self, _ctx, v, n, root):
        import torch
        a = _u64(v, n)
        t = torch.from_numpy(a.view(np.int64).copy())
        self.dist.broadcast(t, src=root, group=self.group)
        a[:] = t.numpy().view(np.uint64)

    def alltoallv(self, _ctx, send, send_off, send_bytes, recv, recv_off, recv_bytes):
        import torch
        W = self.size
        so, sb = _u64(send_off, W), _u64(send_bytes, W)
        ro, rb = _u64(recv_off, W), _u64(recv_bytes, W)
        stot, rtot = int(sb.sum()), int(rb.sum())
        s = np.ctypeslib.as_array(send, shape=(max(1, int(so[-1] + sb[-1])),))
        sendbuf = np.concatenate([s[int(so[p]):int(so[p] + sb[p])] for p in range(W)]) if stot else \
            np.zeros(0, np.uint8)
        out = torch.empty(rtot, dtype=torch.uint8)
        self.dist.all_to_all_single(out, torch.from_numpy(sendbuf.copy()), [int(x) for x in rb],
                                    [int(x) for x in sb], group=self.group)
        r = np.ctypeslib.as_array(recv, shape=(max(1, int(ro[-1] + rb[-1])),))
        o = out.numpy()
        pos = 0
        for p in range(W):
            r[int(ro[p]):int(ro[p] + rb[p])] = o[pos:pos + int(rb[p])]
            pos += int(rb[p])


def comm_unique_id() -> bytes:
    lib = _lib.load()
    buf = (ctypes.c_uint8 * 128)()
    _lib.check(lib.dsl_comm_unique_id(buf), "dsl_comm_unique_id")
    return bytes(buf)


def broadcast_comm_id(rank: int, group=None) -> bytes:
    """Rank 0 makes the RCCL unique id; torch.distributed broadcasts it (plumbing only)."""
    import torch.distributed as dist
    obj = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


def sharded_engine(protocol, host_comm: Optional[TorchHostComm] = None, comm_id: Optional[bytes] = None,
                   device: int = -1):
    """Engine for this process's shard: over RCCL (comm_id) or a caller transport (host_comm)."""
    from .search import Engine
    import torch.distributed as dist
    return Engine(protocol, device=device, rank=dist.get_rank(), world_size=dist.get_world_size(),
                  comm_id=comm_id, host_comm=host_comm)
