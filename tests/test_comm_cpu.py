"""CPU checks of the native sharding's host-side surface (include/dips_hip.h
dips_comm_* / dips_shard_*, shard_abi.hip) -- no device calls: the frame
ranges, the argument checks every communicator constructor makes before it
touches a device, the error record, and the Python wrappers' refusals.
The GPU tests (tests/test_gpu_shard_native.py) run the transports."""
import ctypes

import pytest

from dips_amd import _lib
from dips_amd.comm import Comm, TorchHostTransport, shard_range


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.parametrize("n,g", [(40000, 8), (10000, 8), (37, 2), (67, 8), (5, 5), (7, 3), (0, 4), (2**34 + 3, 8)])
def test_shard_range_partitions(n, g):
    """[r*N/G, (r+1)*N/G): contiguous, covering, balanced to within one frame
    (SURVEY.md s8e), the same as dips_amd.shard.frame_range."""
    from dips_amd import shard
    ranges = [shard_range(n, g, r) for r in range(g)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a, b), (c, _) in zip(ranges, ranges[1:]):
        assert b == c
    sizes = [b - a for a, b in ranges]
    assert max(sizes) - min(sizes) <= 1
    assert ranges == [shard.frame_range(n, g, r) for r in range(g)]


def test_shard_range_refuses_bad_ranks():
    lib = _lib.load()
    first, count = ctypes.c_uint64(), ctypes.c_uint32()
    for g, r in ((0, 0), (4, 4), (4, -1)):
        assert lib.dips_shard_range(10, g, r, ctypes.byref(first), ctypes.byref(count)) == _lib.DIPS_ERR_INVALID
    # a range of 2^32 frames or more does not fit the count
    assert lib.dips_shard_range(1 << 33, 1, 0, ctypes.byref(first), ctypes.byref(count)) == _lib.DIPS_ERR_INVALID


def test_comm_constructors_check_arguments_first():
    lib = _lib.load()
    out = ctypes.c_void_p()
    uid = (ctypes.c_uint8 * 128)()
    assert lib.dips_comm_create(uid, 0, 0, 0, ctypes.byref(out)) == _lib.DIPS_ERR_INVALID
    assert lib.dips_comm_create(uid, 2, 2, 0, ctypes.byref(out)) == _lib.DIPS_ERR_INVALID
    assert lib.dips_comm_create(None, 1, 0, 0, ctypes.byref(out)) == _lib.DIPS_ERR_INVALID
    assert b"rank outside" in lib.dips_comm_last_error(None)
    assert lib.dips_comm_create(uid, 1, 0, 0, None) == _lib.DIPS_ERR_INVALID
    arr = (ctypes.c_void_p * 2)()
    assert lib.dips_comm_create_loopback(0, 0, arr) == _lib.DIPS_ERR_INVALID
    assert lib.dips_comm_create_all(0, None, arr) == _lib.DIPS_ERR_INVALID
    assert lib.dips_comm_create_all(2, None, None) == _lib.DIPS_ERR_INVALID
    assert lib.dips_comm_create_loopback(2, 0, None) == _lib.DIPS_ERR_INVALID
    ops = _lib.DipsCommOps()  # no callbacks
    assert lib.dips_comm_create_host(ctypes.byref(ops), None, 2, 0, 0, ctypes.byref(out)) == _lib.DIPS_ERR_INVALID
    assert b"every callback is required" in lib.dips_comm_last_error(None)
    assert not out.value
    # null communicators are refused, never dereferenced
    lib.dips_comm_destroy(None)
    assert lib.dips_comm_info(None, None, None, None) == _lib.DIPS_ERR_INVALID
    assert lib.dips_diff_series_sharded(None, None, 1, 1, None, 1, 1, None, 0, None, None) == _lib.DIPS_ERR_INVALID
    assert lib.dips_shard_plan(None, None, 1, 1, 1, None, None, None, None) == _lib.DIPS_ERR_INVALID
    assert lib.dips_shard_reference(None, None, 0) == _lib.DIPS_ERR_INVALID
    assert lib.dips_shard_broadcast(None, None, 1, 1, None, None) == _lib.DIPS_ERR_INVALID


@pytest.mark.skipif(_has_gpu(), reason="the no-device error path")
def test_comm_without_device_fails_cleanly():
    from dips_amd import DipsError
    with pytest.raises(DipsError) as ei:
        Comm.loopback(2, 0)
    assert ei.value.status == _lib.DIPS_ERR_NODEVICE and "no HIP device" in str(ei.value)
    with pytest.raises(DipsError) as ei:
        Comm.host(TorchHostTransport(), 2, 0, 0)
    assert ei.value.status == _lib.DIPS_ERR_NODEVICE
    with pytest.raises(ValueError):
        Comm.rccl(b"short", 1, 0, 0)


def test_error_code_and_abi():
    """DIPS_ERR_COMM (-8) in every binding; ABI 3 carries the sharding."""
    assert _lib.DIPS_ERR_COMM == -8 and _lib.ABI_VERSION == 3
    hdr = open(_lib.HEADER_PATH).read()
    assert "DIPS_ERR_COMM = -8" in hdr and "#define DIPS_COMM_ID_BYTES 128u" in hdr
    assert _lib.COMM_ID_BYTES == 128


def _uid_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    from dips_amd import comm as comm_mod
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def no_uid():
            raise _lib.DipsError(_lib.DIPS_ERR_COMM, "bootstrap unavailable")
        comm_mod.Comm.unique_id = staticmethod(no_uid)  # rank 0 cannot make the id
        try:
            comm_mod.rccl_from_process_group(0)
            q.put((rank, "returned"))
        except _lib.DipsError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_rccl_from_process_group_fails_on_every_rank():
    """Rank 0 failing to make the unique id raises on every rank instead of
    leaving the others in the broadcast (gloo, 2 processes, no device)."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_uid_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=120) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all("no RCCL unique id" in got[r] and "bootstrap unavailable" in got[r] for r in range(2)), got
