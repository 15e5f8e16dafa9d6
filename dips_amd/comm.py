"""Communicators of the native sharded series (include/dips_hip.h dips_comm_*).

The frame-range sharding of the difference series lives in libdips_hip.so
(shard_abi.hip: dips_diff_series_sharded -- reference broadcast, halo
send/recv beside the series launch, one gather of the series); this module
only creates the communicator it runs over:

  Comm.rccl(uid, nranks, rank, device)   RCCL over xGMI, one process per GPU
                                         (uid from Comm.unique_id() on rank 0,
                                         handed to the others out of band --
                                         rccl_from_process_group does that over
                                         an initialised torch process group);
  Comm.rccl_all(devices)                 every rank in this process, one
                                         thread per rank (ncclCommInitAll);
  Comm.loopback(nranks, device)          ranks as threads of this process on
                                         one device (tests);
  Comm.host(transport, nranks, rank, device)
                                         the caller's own transport over host
                                         buffers -- TorchHostTransport runs it
                                         over a torch.distributed group (the
                                         gloo rehearsal of bench.py's N > 1
                                         path on one GPU).

The reference is single-device (dips/src/gpu/mod.rs:66-98, adapter request
:71-78); SURVEY.md s8e specifies the sharding.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import check_comm


class Comm:
    """One rank's communicator (dips_comm*)."""

    def __init__(self, ptr: ctypes.c_void_p, keep=None):
        self._lib = _lib.load()
        self._c = ptr
        self._keep = keep  # the host transport's callbacks live as long as the comm
        kind, n, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check_comm(self._lib.dips_comm_info(ptr, ctypes.byref(kind), ctypes.byref(n), ctypes.byref(r)), ptr)
        self.kind, self.nranks, self.rank = kind.value, n.value, r.value

    @property
    def ptr(self) -> ctypes.c_void_p:
        if self._c is None:
            raise _lib.DipsError(_lib.DIPS_ERR_STATE, "communicator destroyed")
        return self._c

    # -- creation ------------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        """A new RCCL unique id (rank 0 makes it, every rank joins with it)."""
        lib = _lib.load()
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        check_comm(lib.dips_comm_unique_id(buf), None)
        return bytes(buf)

    @classmethod
    def rccl(cls, uid: bytes, nranks: int, rank: int, device: int) -> "Comm":
        """Join the RCCL communicator `uid` (ncclCommInitRank; blocks until
        every rank has joined)."""
        lib = _lib.load()
        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError(f"an RCCL unique id has {_lib.COMM_ID_BYTES} bytes")
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        c = ctypes.c_void_p()
        check_comm(lib.dips_comm_create(buf, int(nranks), int(rank), int(device), ctypes.byref(c)), None)
        return cls(c)

    @classmethod
    def rccl_all(cls, devices: List[int]) -> List["Comm"]:
        """Every rank of an RCCL communicator in THIS process
        (ncclCommInitAll), rank r on devices[r]; drive each from its own
        thread."""
        lib = _lib.load()
        n = len(devices)
        devs = (ctypes.c_int * n)(*[int(d) for d in devices])
        arr = (ctypes.c_void_p * n)()
        check_comm(lib.dips_comm_create_all(n, devs, arr), None)
        return [cls(ctypes.c_void_p(p)) for p in arr]

    @classmethod
    def loopback(cls, nranks: int, device: int = 0) -> List["Comm"]:
        """`nranks` loopback ranks on `device`; drive each from its own thread."""
        lib = _lib.load()
        arr = (ctypes.c_void_p * int(nranks))()
        check_comm(lib.dips_comm_create_loopback(int(nranks), int(device), arr), None)
        return [cls(ctypes.c_void_p(p)) for p in arr]

    @classmethod
    def host(cls, transport, nranks: int, rank: int, device: int) -> "Comm":
        """A communicator over `transport`, an object with
        broadcast(buf, root), sendrecv(send, to, recv, src) and
        gather(send, recv, root) on numpy uint8 arrays (None where a side is
        absent); an exception in any of them fails the sharded call with
        DIPS_ERR_COMM."""
        lib = _lib.load()

        def view(ptr, n):
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(n,)) if ptr else None

        def bcast(_ctx, buf, nbytes, root):
            try:
                transport.broadcast(view(buf, nbytes), root)
                return 0
            except Exception:  # reported to the library as a failure code
                return 1

        def sendrecv(_ctx, send, to, recv, src, nbytes):
            try:
                transport.sendrecv(view(send, nbytes), to, view(recv, nbytes), src)
                return 0
            except Exception:
                return 1

        def gather(_ctx, send, recv, nbytes, root):
            try:
                transport.gather(view(send, nbytes), view(recv, nbytes * nranks), root)
                return 0
            except Exception:
                return 1

        ops = _lib.DipsCommOps(_lib.COMM_BROADCAST_FN(bcast), _lib.COMM_SENDRECV_FN(sendrecv),
                               _lib.COMM_GATHER_FN(gather))
        c = ctypes.c_void_p()
        check_comm(lib.dips_comm_create_host(ctypes.byref(ops), None, int(nranks), int(rank), int(device),
                                             ctypes.byref(c)), None)
        return cls(c, keep=ops)

    # -- lifetime ------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_c", None) is not None:
            self._lib.dips_comm_destroy(self._c)
            self._c = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __repr__(self) -> str:
        kind = {_lib.COMM_RCCL: "rccl", _lib.COMM_LOOPBACK: "loopback", _lib.COMM_HOST: "host"}.get(self.kind, "?")
        return f"Comm({kind}, rank {self.rank} of {self.nranks})"


def shard_range(n_total: int, nranks: int, rank: int):
    """[first, first + count) of `rank` (dips_shard_range)."""
    lib = _lib.load()
    first, count = ctypes.c_uint64(), ctypes.c_uint32()
    if lib.dips_shard_range(int(n_total), int(nranks), int(rank), ctypes.byref(first), ctypes.byref(count)) != 0:
        raise ValueError("bad shard range")
    return first.value, first.value + count.value


class TorchHostTransport:
    """DIPS_COMM_HOST over a torch.distributed group whose backend moves host
    tensors (gloo): the transport of bench.py's N > 1 rehearsal, where the
    ranks share one GPU and RCCL refuses them ("Duplicate GPU detected")."""

    def __init__(self, group=None):
        self.group = group

    def broadcast(self, buf, root):
        import torch
        import torch.distributed as dist
        dist.broadcast(torch.from_numpy(buf), src=root, group=self.group)

    def sendrecv(self, send, to, recv, src):
        import torch
        import torch.distributed as dist
        ops = []
        if send is not None and to >= 0:
            ops.append(dist.P2POp(dist.isend, torch.from_numpy(send), to, self.group))
        if recv is not None and src >= 0:
            ops.append(dist.P2POp(dist.irecv, torch.from_numpy(recv), src, self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()

    def gather(self, send, recv, root):
        import torch
        import torch.distributed as dist
        t = torch.from_numpy(send)
        if dist.get_rank(self.group) == root:
            parts = list(torch.from_numpy(recv).view(-1, send.size).unbind(0))
            dist.gather(t, gather_list=parts, dst=root, group=self.group)
        else:
            dist.gather(t, dst=root, group=self.group)


def rccl_from_process_group(device: int, group=None) -> Comm:
    """The RCCL communicator of an initialised torch process group's ranks:
    rank 0's unique id travels over the group (broadcast_object_list).  If
    rank 0 cannot make one, every rank raises (none is left waiting in the
    broadcast or in ncclCommInitRank)."""
    import torch.distributed as dist
    msg: List[Optional[object]] = [None, None]  # [unique id, rank 0's error]
    if dist.get_rank(group) == 0:
        try:
            msg[0] = Comm.unique_id()
        except Exception as e:  # travels to every rank, raised there
            msg[1] = f"{type(e).__name__}: {e}"
    dist.broadcast_object_list(msg, src=0, group=group)
    if msg[0] is None:
        raise _lib.DipsError(_lib.DIPS_ERR_COMM, f"rank 0 made no RCCL unique id ({msg[1]})")
    return Comm.rccl(msg[0], dist.get_world_size(group), dist.get_rank(group), device)


__all__ = ["Comm", "TorchHostTransport", "rccl_from_process_group", "shard_range"]
