"""The frame-range sharded series (dips_amd.shard) with the HIP operator as
the per-rank compute: two processes on the one GPU of the box, gloo as the
process group (RCCL refuses two ranks on one device, "Duplicate GPU
detected"), the halo frame and the series staged through host tensors since
gloo has no device send/recv.  Each rank runs DiffSeriesOperator.run_device
on its shard; the gathered series must equal one single-process launch over
all frames.  The last test runs the
native sharded call (dips_diff_series_sharded) in the same two processes over
the DIPS_COMM_HOST transport backed by the gloo group."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

W, H, SEED = 256, 96, 0xD1B5
TAU = 8 / 255


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _hip_compute(op):
    """compute(frames, ref, series_out) over host tensors: upload, run the
    HIP series kernel, download (the shard protocol's tensors stay on the
    host for gloo)."""
    def compute(frames, ref, series_out):
        dev = frames.cuda()
        rdev = ref.cuda() if ref is not None else None
        ser = torch.zeros((frames.shape[0], 4), dtype=torch.int64, device="cuda")
        op.run_device(dev, ser, ref=rdev)
        torch.cuda.synchronize()
        series_out.copy_(ser.cpu())
    return compute


def _worker(rank, world, port, n_total, mode, overlapped, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = None
    try:
        from dips_amd import DiffSeriesOperator, Mode, PixelFormat, shard
        torch.cuda.set_device(0)
        s, e = shard.frame_range(n_total, world, rank)
        # this rank's frames generated on the device by the shared generator
        op = DiffSeriesOperator(PixelFormat.RGB8, Mode(mode), TAU)
        dev = torch.empty((e - s, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(dev, W, H, SEED, s)
        torch.cuda.synchronize()
        local = dev.cpu()
        compute = _hip_compute(op)
        if mode == 0:
            ref = local[0].clone() if rank == 0 else torch.empty_like(local[0])
            shard.broadcast_reference(ref)
            full = shard.sharded_series(local, per_frame=False, n_total=n_total, compute=compute, reference=ref)
        elif overlapped:
            series = torch.zeros((local.shape[0], shard.SERIES_COLS), dtype=torch.int64)
            shard.per_frame_overlapped(local, torch.empty_like(local[0]), series, compute)
            full = shard.SeriesGather(n_total, torch.device("cpu"))(series)
        else:
            full = shard.sharded_series(local, per_frame=True, n_total=n_total, compute=compute)
        if rank == 0:
            result_q.put(full.numpy().copy())
    finally:
        if op is not None:
            op.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,overlapped", [(0, False), (1, False), (1, True)])
def test_sharded_hip_equals_single_launch(mode, overlapped):
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    world, n_total = 2, 37
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, mode, overlapped, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    # one single-process launch over all frames (no wave cap)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode(mode), TAU)
    try:
        allf = torch.empty((n_total, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(allf, W, H, SEED, 0)
        one = torch.zeros((n_total, 4), dtype=torch.int64, device="cuda")
        op.run_device(allf, one, ref=None if mode == 1 else allf[0])
        torch.cuda.synchronize()
    finally:
        op.close()
    want = one.cpu().numpy()
    assert got.shape == want.shape
    assert np.array_equal(got, want)
    assert want[:, 0].any()  # non-trivial series


def _verify_worker(rank, world, port, n_total, mode, corrupt, result_q):
    """The bench's N > 1 step with the HIP operator, then its self-check
    (shard.verify_sharded_series) with the HIP operator regenerating frames
    on the device; `corrupt` = "halo" damages rank 1's received halo."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = None
    try:
        from dips_amd import DiffSeriesOperator, Mode, PixelFormat, shard
        torch.cuda.set_device(0)
        s, e = shard.frame_range(n_total, world, rank)
        op = DiffSeriesOperator(PixelFormat.RGB8, Mode(mode), TAU)
        dev = torch.empty((e - s, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(dev, W, H, SEED, s)
        torch.cuda.synchronize()
        local = dev.cpu()
        hip = _hip_compute(op)

        def compute(fr, r, out):
            if corrupt == "halo" and rank == 1 and r is not None and fr.shape[0] == 1:
                r[7, 9, 2] ^= 0x33
            hip(fr, r, out)

        ref = torch.empty_like(local[0])
        series = torch.zeros((e - s, shard.SERIES_COLS), dtype=torch.int64)
        if mode == 0:
            if rank == 0:
                ref.copy_(local[0])
            shard.broadcast_reference(ref)
            compute(local, ref, series)
        else:
            shard.per_frame_overlapped(local, ref, series, compute)
        full = shard.SeriesGather(n_total, torch.device("cpu"))(series)
        chk = shard.verify_sharded_series(op, width=W, height=H, seed=SEED, n_total=n_total,
                                          per_frame=(mode == 1), local_series=series, ref=ref,
                                          gathered=full, device=torch.device("cuda", 0))
        torch.cuda.synchronize()
        result_q.put((rank, chk))
    finally:
        if op is not None:
            op.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,corrupt", [(1, None), (0, None), (1, "halo")])
def test_bench_self_check(mode, corrupt):
    """bench.py's N > 1 self-check with the HIP operator in two processes:
    equal on a correct step, not equal on every rank when the halo is
    damaged."""
    from dips_amd import shard
    world, n_total = 2, 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, n_total, mode, corrupt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = sorted(q.get(timeout=300) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    for _, chk in got:
        assert chk["equal"] is (corrupt is None), chk
        assert chk["frames_checked"] >= len(shard.check_frames(n_total, world))


def _native_worker(rank, world, port, n_total, mode, host_ptrs, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    op = comm = None
    try:
        from dips_amd import DiffSeriesOperator, Mode, PixelFormat
        from dips_amd.comm import Comm, TorchHostTransport, shard_range
        torch.cuda.set_device(0)
        s, e = shard_range(n_total, world, rank)
        op = DiffSeriesOperator(PixelFormat.RGB8, Mode(mode), TAU)
        comm = Comm.host(TorchHostTransport(), world, rank, 0)
        dev = torch.empty((e - s, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(dev, W, H, SEED, s)
        torch.cuda.synchronize()
        if host_ptrs:
            _, full = op.sharded(comm, dev.cpu().numpy(), n_total)
            full = full.as_array() if full is not None else None
        else:
            loc = torch.zeros((e - s, 4), dtype=torch.int64, device="cuda")
            all_ = torch.zeros((n_total, 4), dtype=torch.int64, device="cuda") if rank == 0 else None
            op.run_sharded(comm, dev, n_total, loc, all_)
            torch.cuda.synchronize()
            full = all_.cpu().numpy().view(np.uint64) if rank == 0 else None
        if rank == 0:
            result_q.put(full.copy())
    finally:
        if op is not None:
            op.close()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,host_ptrs", [(2, 0, False), (2, 1, False), (2, 1, True), (3, 1, False),
                                                   (3, 0, True)])
def test_native_sharded_over_host_transport(world, mode, host_ptrs):
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    n_total = 33
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_worker, args=(r, world, port, n_total, mode, host_ptrs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode(mode), TAU)
    try:
        allf = torch.empty((n_total, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(allf, W, H, SEED, 0)
        one = torch.zeros((n_total, 4), dtype=torch.int64, device="cuda")
        op.run_device(allf, one)
        torch.cuda.synchronize()
    finally:
        op.close()
    assert np.array_equal(got, one.cpu().numpy().view(np.uint64))


def _alt_frames(n):
    rng = np.random.default_rng(505)
    return rng.integers(0, 256, (n, 24, 40, 4), dtype=np.uint8)


ALT_MARKERS = [6, 11, 12, 20]


def _native_alt_worker(rank, world, port, n_total, host_ptrs, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    runner = comm = None
    try:
        from dips_amd.alt import DiPsRunner
        from dips_amd.comm import Comm, TorchHostTransport, shard_range
        torch.cuda.set_device(0)
        s, e = shard_range(n_total, world, rank)
        frames = _alt_frames(n_total)[s:e]
        runner = DiPsRunner(24, 40, refresh_markers=ALT_MARKERS)
        comm = Comm.host(TorchHostTransport(), world, rank, 0)
        if host_ptrs:
            out = runner.run_sharded(comm, frames, n_total)
        else:
            dev = torch.from_numpy(frames).cuda()
            o = torch.empty_like(dev)
            runner.run_sharded_device(comm, dev, o, n_total)
            out = o.cpu().numpy()
        result_q.put((rank, out))
    finally:
        if runner is not None:
            runner.close()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,host_ptrs", [(2, True), (3, False)])
def test_native_alt_sharded_over_host_transport(world, host_ptrs):
    """dips_alt_run_sharded in `world` processes over DIPS_COMM_HOST (gloo):
    the ranks' outputs equal one run_dips_on_file loop over every frame."""
    from dips_amd.alt import DiPsRunner
    n_total = 26
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_alt_worker, args=(r, world, port, n_total, host_ptrs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = dict(q.get(timeout=300) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    frames = _alt_frames(n_total)
    r = DiPsRunner(24, 40, refresh_markers=ALT_MARKERS)
    try:
        want = r(frames)
    finally:
        r.close()
    assert np.array_equal(np.concatenate([parts[k] for k in range(world)]), want)


def _native_compat_worker(rank, world, port, n_total, host_ptrs, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cs = comm = None
    try:
        from dips_amd import ChromaFilter, ComputeState, DiPsFilter
        from dips_amd.comm import Comm, TorchHostTransport, shard_range
        torch.cuda.set_device(0)
        s, e = shard_range(n_total, world, rank)
        frames = _alt_frames(n_total)[s:e]
        cs = ComputeState(True, 3, 4.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
        comm = Comm.host(TorchHostTransport(), world, rank, 0)
        if host_ptrs:
            out = cs.frame_callback_batch_sharded(comm, 40, 24, frames, n_total)
        else:
            dev = torch.from_numpy(frames).cuda()
            o = torch.empty_like(dev)
            cs.frame_callback_batch_sharded_device(comm, dev, o, n_total)
            torch.cuda.synchronize()
            out = o.cpu().numpy()
        result_q.put((rank, out))
    finally:
        if cs is not None:
            cs.close()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,host_ptrs", [(2, False), (3, True)])
def test_native_compat_sharded_over_host_transport(world, host_ptrs):
    """dips_frame_callback_batch_sharded in `world` processes over
    DIPS_COMM_HOST (gloo), window 3: the ranks' outputs equal one
    ComputeState's frame_callback_batch over every frame."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    n_total = 26
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_compat_worker, args=(r, world, port, n_total, host_ptrs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        parts = dict(q.get(timeout=300) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    cs = ComputeState(True, 3, 4.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    try:
        want = cs.frame_callback_batch(40, 24, _alt_frames(n_total))
    finally:
        cs.close()
    assert np.array_equal(np.concatenate([parts[k] for k in range(world)]), want)
