"""World-size-2 gloo tests of the frame-range sharding protocol
(dips_amd.shard): halo exchange, reference broadcast and the single series
gather reassemble exactly the single-process series.  The per-rank compute
here is the CPU oracle (test seam); on GPUs it is the HIP operator."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dips_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_compute(mode, tau):
    from oracle import oracle

    def compute(frames, ref, series_out):
        f = frames.numpy()
        r = ref.numpy() if ref is not None else None
        out4, _, _ = oracle.series(f, mode=mode, tau=tau, ref=r)
        series_out.copy_(torch.from_numpy(out4.view(np.int64)))
    return compute


def _worker(rank, world, port, n_total, mode, tau, result_q, overlapped=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        all_frames = oracle.synth(3, 32, 16, 5, 0, n_total)
        s, e = shard.frame_range(n_total, world, rank)
        local = torch.from_numpy(all_frames[s:e].copy())
        reference = None
        if mode == 0:
            reference = torch.from_numpy(all_frames[0].copy()) if rank == 0 else torch.empty_like(local[0])
            shard.broadcast_reference(reference)
        if overlapped:
            # bench.py's per-frame step: halo transfer behind frames 1..n-1
            series = torch.zeros((local.shape[0], shard.SERIES_COLS), dtype=torch.int64)
            halo = torch.empty_like(local[0])
            shard.per_frame_overlapped(local, halo, series, _oracle_compute(mode, tau))
            full = shard.SeriesGather(n_total, torch.device("cpu"))(series)
        else:
            full = shard.sharded_series(local, per_frame=(mode == 1), n_total=n_total,
                                        compute=_oracle_compute(mode, tau), reference=reference)
        if rank == 0:
            result_q.put(full.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,overlapped", [(0, False), (1, False), (1, True)])
@pytest.mark.parametrize("n_total", [7, 8])
def test_sharded_equals_single(mode, overlapped, n_total):
    from oracle import oracle
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, mode, 2 / 255, q, overlapped))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    frames = oracle.synth(3, 32, 16, 5, 0, n_total)
    want, _, _ = oracle.series(frames, mode=mode, tau=2 / 255)
    assert np.array_equal(got.view(np.uint64), want)


def test_frame_ranges_cover_and_balance():
    for n in (1, 7, 40000):
        for world in (1, 2, 3, 8):
            r = shard.frame_ranges(n, world)
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            sizes = [e - s for s, e in r]
            assert max(sizes) - min(sizes) <= 1


def _compat_worker(rank, world, port, n_total, params, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        w, h = 20, 12
        rng = np.random.default_rng(77)
        allf = rng.integers(0, 256, (n_total, h, w, 4), dtype=np.uint8)
        s, e = shard.frame_range(n_total, world, rank)
        local = torch.from_numpy(allf[s:e].copy())
        cs = oracle.ComputeState(*params)

        def callback_batch(fr):
            return torch.from_numpy(np.stack([oracle.frame_callback(w, h, f, cs) for f in fr.numpy()]))

        def start_texture(buf):
            buf.copy_(torch.from_numpy(cs.start_texture()))

        def resume(start, halo, t0):
            cs.resume(w, h, start.numpy(), halo.numpy(), t0)

        out = shard.compat_sharded(local, s, callback_batch=callback_batch, start_texture=start_texture,
                                   resume=resume, start_buf=torch.zeros((h, w, 4), dtype=torch.uint8),
                                   halo_buf=torch.zeros((3, h, w, 4), dtype=torch.uint8))
        # reassemble on rank 0 (padded gather; the product keeps outputs per rank)
        m = max(b - a for a, b in shard.frame_ranges(n_total, world))
        pad = torch.zeros((m, h, w, 4), dtype=torch.uint8)
        pad[: out.shape[0]] = out
        bufs = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
        dist.gather(pad, bufs, dst=0)
        if rank == 0:
            full = torch.cat([b[: e2 - s2] for b, (s2, e2) in zip(bufs, shard.frame_ranges(n_total, world))])
            result_q.put(full.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,params", [(2, 24, (True, 1, 5.0, 0, 0)), (3, 40, (False, 1, 0.7, 255, 2)),
                                                  (2, 31, (True, 3, 5.0, 1, 0))])
def test_compat_sharded_equals_single(world, n_total, params):
    """dips-compat frame_callback over frame ranges (start texture broadcast
    + 3-frame halo + resume) gives the single ComputeState's outputs."""
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_compat_worker, args=(r, world, port, n_total, params, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w, h = 20, 12
    frames = np.random.default_rng(77).integers(0, 256, (n_total, h, w, 4), dtype=np.uint8)
    cs = oracle.ComputeState(*params)
    want = np.stack([oracle.frame_callback(w, h, f, cs) for f in frames])
    assert np.array_equal(got, want)


def test_alt_run_loop_flags_match_oracle_loop():
    """alt.run_loop_flags restates run_dips_on_file's snapshot schedule: one
    oracle DiPsCompute fed frame by frame with those flags gives the oracle
    run loop's outputs."""
    from oracle import oracle
    from dips_amd.alt import run_loop_flags
    w, h, n = 12, 8, 30
    frames = np.random.default_rng(5).integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    for markers in ([], [3], [5, 6, 19], [1, 2, 3, 28]):
        flags = run_loop_flags(n, markers)
        a = oracle.AltCompute(2, w, h)
        got = np.stack([a.send_frame(frames[t], bool(flags[t])) for t in range(n)])
        want = oracle.AltCompute(2, w, h).run(frames, markers)
        assert np.array_equal(got, want), markers


def _alt_worker(rank, world, port, n_total, n_tex, markers, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        from dips_amd.alt import run_loop_flags
        w, h = 14, 10
        allf = np.random.default_rng(31).integers(0, 256, (n_total, h, w, 4), dtype=np.uint8)
        s, e = shard.frame_range(n_total, world, rank)
        local = torch.from_numpy(allf[s:e].copy())
        flags = run_loop_flags(n_total, markers)
        comp = oracle.AltCompute(n_tex, w, h, True, 1, 5.0, 0, 0)

        def send_frames(fr, fl):
            return torch.from_numpy(np.stack([comp.send_frame(f, bool(x)) for f, x in zip(fr.numpy(), fl)]))

        out = shard.alt_sharded(local, s, n_total, flags, n_tex, send_frames=send_frames)
        m = max(b - a for a, b in shard.frame_ranges(n_total, world))
        pad = torch.zeros((m, h, w, 4), dtype=torch.uint8)
        pad[: out.shape[0]] = out
        bufs = [torch.zeros_like(pad) for _ in range(world)] if rank == 0 else None
        dist.gather(pad, bufs, dst=0)
        if rank == 0:
            full = torch.cat([b[: e2 - s2] for b, (s2, e2) in zip(bufs, shard.frame_ranges(n_total, world))])
            result_q.put(full.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,n_tex,markers", [(2, 20, 2, [5, 6]), (3, 31, 3, [9, 10, 22]),
                                                        (3, 12, 2, [2, 3, 4, 5, 6, 7, 8, 9, 10, 11]),
                                                        # N > t0 + 1: zero slots still live at the shard
                                                        # start, a snapshot before it
                                                        (2, 10, 16, []), (3, 14, 6, [1]), (2, 9, 5, [])])
def test_alt_sharded_equals_single(world, n_total, n_tex, markers):
    """dips_alt run loop over frame ranges (the last snapshot's source frames
    and an N-frame halo replayed into a fresh DiPsCompute) gives the single
    loop's outputs, snapshots falling on and across shard edges."""
    from oracle import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_alt_worker, args=(r, world, port, n_total, n_tex, markers, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w, h = 14, 10
    frames = np.random.default_rng(31).integers(0, 256, (n_total, h, w, 4), dtype=np.uint8)
    want = oracle.AltCompute(n_tex, w, h, True, 1, 5.0, 0, 0).run(frames, markers)
    assert np.array_equal(got, want)


def _compat_bad_worker(rank, world, port, n_total, result_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, h = 8, 4
        s, e = shard.frame_range(n_total, world, rank)
        local = torch.zeros((e - s, h, w, 4), dtype=torch.uint8)
        try:
            shard.compat_sharded(local, s, callback_batch=lambda fr: fr, start_texture=lambda b: None,
                                 resume=lambda *a: None, start_buf=torch.zeros((h, w, 4), dtype=torch.uint8),
                                 halo_buf=torch.zeros((3, h, w, 4), dtype=torch.uint8))
            result_q.put((rank, "no error"))
        except ValueError as ex:
            result_q.put((rank, str(ex)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total", [(2, 8), (3, 20)])
def test_compat_sharded_bad_layout_fails_on_every_rank(world, n_total):
    """A shard layout the dips-compat resume cannot take (a rank starting
    before global frame 7) raises the same ValueError on every rank instead
    of leaving the others blocked in the halo exchange."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_compat_bad_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r, _ in got] == list(range(world))
    msgs = {m for _, m in got}
    assert len(msgs) == 1 and "frame >= 7" in msgs.pop()


class _OracleOp:
    """CPU stand-in for DiffSeriesOperator's device calls (test seam for
    shard.verify_sharded_series): synth_device / run_device on host tensors
    through the oracle."""

    def __init__(self, mode, tau, channels=3):
        from dips_amd import PixelFormat
        self.fmt = PixelFormat(channels)
        self.mode, self.tau = mode, tau

    def synth_device(self, dst, width, height, seed, t0):
        from oracle import oracle
        dst.copy_(torch.from_numpy(oracle.synth(int(self.fmt), width, height, seed, t0, dst.shape[0])))

    def run_device(self, frames, out, ref=None):
        from oracle import oracle
        out4, _, _ = oracle.series(frames.numpy(), mode=self.mode, tau=self.tau,
                                   ref=ref.numpy() if ref is not None else None)
        out.copy_(torch.from_numpy(out4.view(np.int64)))


def _verify_worker(rank, world, port, n_total, mode, corrupt, result_q):
    """bench.py's N > 1 step (broadcast or overlapped halo + one gather) then
    its self-check; `corrupt` damages one exchange on purpose."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W, H, SEED, tau = 32, 16, 5, 2 / 255
        op = _OracleOp(mode, tau)
        s, e = shard.frame_range(n_total, world, rank)
        local = torch.empty((e - s, H, W, 3), dtype=torch.uint8)
        op.synth_device(local, W, H, SEED, s)
        ref = torch.empty_like(local[0])
        series = torch.zeros((e - s, shard.SERIES_COLS), dtype=torch.int64)

        def compute(fr, r, out):
            if corrupt == "halo" and rank == 1 and r is not None and fr.shape[0] == 1:
                r[3, 5, 1] ^= 0x5A  # the received halo damaged before frame 0 uses it
            op.run_device(fr, out, ref=r)

        if mode == 0:
            if rank == 0:
                ref.copy_(local[0])
            shard.broadcast_reference(ref)
            if corrupt == "ref" and rank == world - 1:
                ref[0, 0, 0] ^= 0x01
            compute(local, ref, series)
        else:
            shard.per_frame_overlapped(local, ref, series, compute)
        full = shard.SeriesGather(n_total, torch.device("cpu"))(series)
        if corrupt == "gather" and rank == 0:
            b = shard.frame_range(n_total, world, 1)[0]
            full = full.clone()
            full[[b - 1, b]] = full[[b, b - 1]]  # two rows of a boundary swapped
        chk = shard.verify_sharded_series(op, width=W, height=H, seed=SEED, n_total=n_total,
                                          per_frame=(mode == 1), local_series=series, ref=ref,
                                          gathered=full, device=torch.device("cpu"))
        result_q.put((rank, chk))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_total,mode,corrupt", [
    (2, 9, 1, None), (3, 14, 1, None), (2, 9, 0, None), (3, 14, 0, None),
    (2, 9, 1, "halo"), (3, 14, 1, "gather"), (3, 14, 0, "ref"), (2, 9, 0, "gather")])
def test_verify_sharded_series(world, n_total, mode, corrupt):
    """bench.py's N > 1 self-check passes on a correct sharded step and
    fails, on every rank, when the halo, the broadcast reference or the
    gather is damaged."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, n_total, mode, corrupt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r for r, _ in got] == list(range(world))
    for _, chk in got:
        assert chk["equal"] is (corrupt is None), chk
        assert chk["frames_checked"] >= len(shard.check_frames(n_total, world))
    if corrupt in ("halo", "ref"):
        assert not got[0][1]["local_equal"]
    if corrupt == "gather":
        assert got[0][1]["local_equal"] and not got[0][1]["gathered_equal"]


def test_check_frames_cover_boundaries():
    picks = shard.check_frames(40000, 8)
    for s, _ in shard.frame_ranges(40000, 8)[1:]:
        assert {s - 1, s, s + 1} <= set(picks)
    assert 0 in picks and 39999 in picks and len(picks) >= 2 + 21
