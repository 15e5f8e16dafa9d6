"""The native frame-range sharding (include/dips_hip.h dips_diff_series_sharded,
shard_abi.hip) through the C ABI, on the one GPU of the box:

* RCCL at world size 1 (the RCCL transport's broadcast and gather run; no
  halo at one rank): the sharded call equals dips_diff_series bit for bit,
  device and host pointers, both modes, every format;
* the loopback transport -- ranks as threads of this process on the one
  device -- at world sizes 2, 3 and 8: the gathered series of both modes
  equals one single launch over all frames, and the oracle at every shard
  boundary (get_intensity, dips/src/gpu/shaders/dips_shader.wgsl:64-82);
  every rank's first-frame reference (the halo it received, the broadcast
  reference) equals the frame it must be; ragged shards (n_total not a
  multiple of the world size) take the trimmed gather;
* the plan: the launch beside the halo runs the full persistent grid; the
  DIPS_SERIES_WAVES_PER_SIMD deployment cap, when set, gives fewer waves than
  the uncapped grid (both reported by dips_shard_plan);
* argument errors return on the rank that has them, with the message.

The reference is single-device (dips/src/gpu/mod.rs:71-78); the sharding is
SURVEY.md s8e's."""
import threading

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

SEED, TAU = 0xD1B5, 8.0 / 255.0


def _fmt(name):
    from dips_amd import PixelFormat
    return getattr(PixelFormat, name)


def _shape(c, h, w):
    return (h, w) if c == 1 else (h, w, c)


def _single_launch(fmt_name, mode, n_total, w, h, tau=TAU):
    """One dips_diff_series over all n_total frames (and the frames)."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode
    fmt = _fmt(fmt_name)
    c = int(fmt)
    op = DiffSeriesOperator(fmt, Mode(mode), tau)
    try:
        allf = torch.empty((n_total,) + _shape(c, h, w), dtype=torch.uint8, device="cuda")
        op.synth_device(allf, w, h, SEED, 0)
        one = torch.zeros((n_total, 4), dtype=torch.int64, device="cuda")
        op.run_device(allf, one)
        torch.cuda.synchronize()
        return one.cpu().numpy().view(np.uint64), allf
    finally:
        op.close()


def _run_loopback(world, n_total, fmt_name, mode, w, h, tau=TAU, ref_resident=False, host=False):
    """Every rank of a loopback communicator on its own thread; returns
    (gathered series, [local series], [first-frame reference], plans)."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode
    from dips_amd.comm import Comm, shard_range
    fmt = _fmt(fmt_name)
    c = int(fmt)
    comms = Comm.loopback(world, 0)
    ops = [DiffSeriesOperator(fmt, Mode(mode), tau) for _ in range(world)]
    try:
        ranges = [shard_range(n_total, world, r) for r in range(world)]
        frames = []
        for r, (s, e) in enumerate(ranges):
            f = torch.empty((e - s,) + _shape(c, h, w), dtype=torch.uint8, device="cuda")
            ops[r].synth_device(f, w, h, SEED, s)
            frames.append(f)
        refs = [None] * world
        if ref_resident:  # every rank holds frame 0 already (dips_shard_broadcast's job)
            f0 = torch.empty(_shape(c, h, w), dtype=torch.uint8, device="cuda")
            ops[0].synth_device(f0.unsqueeze(0), w, h, SEED, 0)
            refs = [f0.clone() for _ in range(world)]
        torch.cuda.synchronize()
        local = [torch.zeros((e - s, 4), dtype=torch.int64, device="cuda") for s, e in ranges]
        full = torch.zeros((n_total, 4), dtype=torch.int64, device="cuda")
        got_host = [None] * world
        errors = []

        def rank(r):
            try:
                if host:
                    fr = frames[r].cpu().numpy()
                    got_host[r] = ops[r].sharded(comms[r], fr, n_total,
                                                 ref=refs[r].cpu().numpy() if refs[r] is not None else None,
                                                 ref_resident=ref_resident)
                else:
                    ops[r].run_sharded(comms[r], frames[r], n_total, local[r], full if r == 0 else None,
                                       ref=refs[r], ref_resident=ref_resident)
            except Exception as e:  # reported below
                errors.append((r, repr(e)))

        threads = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=180)
        assert not any(t.is_alive() for t in threads), "a loopback rank did not finish"
        assert not errors, errors
        torch.cuda.synchronize()
        first_refs = []
        for r in range(world):
            out = torch.empty(_shape(c, h, w), dtype=torch.uint8, device="cuda")
            if not host:
                assert ops[r].shard_reference_device(out)
                torch.cuda.synchronize()
                first_refs.append(out.cpu().numpy())
        plans = [ops[r].shard_plan(comms[r], w, h, n_total) for r in range(world)]
        if host:
            full_np = got_host[0][1].as_array()
            local_np = [g[0].as_array() for g in got_host]
        else:
            full_np = full.cpu().numpy().view(np.uint64)
            local_np = [l.cpu().numpy().view(np.uint64) for l in local]
        return full_np, local_np, first_refs, plans, ranges
    finally:
        for o in ops:
            o.close()
        for cm in comms:
            cm.close()


# -- loopback: world sizes 2, 3, 8, both modes ---------------------------------
@pytest.mark.parametrize("world,n_total", [(2, 37), (3, 40), (8, 67), (8, 64)])
@pytest.mark.parametrize("mode", [0, 1])
def test_loopback_equals_single_launch_and_oracle(world, n_total, mode):
    W, H = 320, 96
    full, local, first_refs, plans, ranges = _run_loopback(world, n_total, "RGB8", mode, W, H)
    want, allf = _single_launch("RGB8", mode, n_total, W, H)
    bad = np.nonzero(~np.all(full == want, axis=1))[0]
    assert bad.size == 0, f"gathered rows differing from the single launch: {bad[:10]}"
    for r, (s, e) in enumerate(ranges):
        assert np.array_equal(local[r], want[s:e]), r
    assert want[:, 0].any()
    # the oracle at both sides of every shard boundary (+ the first / last frame)
    frames = allf.cpu().numpy()
    picks = sorted({0, n_total - 1} | {g for s, _ in ranges[1:] for g in (s - 1, s)})
    for g in picks:
        if mode == 1:
            pair = frames[[max(g - 1, 0), g]]
            o, _, _ = oracle.series(pair, mode=1, tau=TAU, nthreads=8)
            row = o[1] if g > 0 else o[0]
        else:
            o, _, _ = oracle.series(frames[[0, g]], mode=0, tau=TAU, nthreads=8)
            row = o[1]
        assert np.array_equal(full[g], row), (g, full[g], row)
    # what each rank's first frame was compared with
    for r, (s, _) in enumerate(ranges):
        want_ref = frames[s - 1] if (mode == 1 and r > 0) else frames[0]
        assert np.array_equal(first_refs[r], want_ref), r
    # the plan: this rank's range; the full grid (no cap set)
    for r, p in enumerate(plans):
        assert (p["first"], p["first"] + p["count"]) == ranges[r]
        assert 0 < p["waves"] == p["waves_uncapped"]


@pytest.mark.parametrize("fmt_name", ["GRAY8", "RGBA8"])
@pytest.mark.parametrize("mode", [0, 1])
def test_loopback_other_formats(fmt_name, mode):
    fmt_name = {"GRAY8": "Gray8", "RGBA8": "RGBA8"}[fmt_name]
    W, H, n_total = 256, 64, 29
    full, _, _, _, _ = _run_loopback(3, n_total, fmt_name, mode, W, H)
    want, _ = _single_launch(fmt_name, mode, n_total, W, H)
    assert np.array_equal(full, want)


def test_loopback_host_pointers_and_resident_reference():
    W, H, n_total = 192, 80, 23
    for mode, resident in ((1, False), (0, False), (0, True)):
        full, local, _, _, ranges = _run_loopback(2, n_total, "RGB8", mode, W, H, ref_resident=resident, host=True)
        want, _ = _single_launch("RGB8", mode, n_total, W, H)
        assert np.array_equal(full, want), (mode, resident)
        for r, (s, e) in enumerate(ranges):
            assert np.array_equal(local[r], want[s:e]), (mode, resident, r)


def test_loopback_part_major_shards_4k(monkeypatch):
    """The bench's shape on 2 loopback ranks: 4K RGB8, 'per-frame', 600
    frames (300 a rank: the part-major schedule; on rank 1 the 299-frame
    launch beside the halo), once on the full grid and once under the
    DIPS_SERIES_WAVES_PER_SIMD=3 deployment cap, which the plan reports as
    fewer waves than the uncapped grid."""
    W, H, n_total = 3840, 2160, 600
    want, _ = _single_launch("RGB8", 1, n_total, W, H)
    full, _, _, plans, _ = _run_loopback(2, n_total, "RGB8", 1, W, H)
    assert np.array_equal(full, want)
    assert plans[1]["waves"] == plans[1]["waves_uncapped"], plans
    monkeypatch.setenv("DIPS_SERIES_WAVES_PER_SIMD", "3")
    full, _, _, plans, _ = _run_loopback(2, n_total, "RGB8", 1, W, H)
    assert np.array_equal(full, want)
    assert 0 < plans[1]["waves"] < plans[1]["waves_uncapped"], plans


# -- RCCL at world size 1 ------------------------------------------------------
@pytest.mark.parametrize("fmt_name", ["RGB8", "RGBA8", "Gray8"])
@pytest.mark.parametrize("mode", [0, 1])
def test_rccl_world1_equals_diff_series(fmt_name, mode):
    import torch
    from dips_amd import DiffSeriesOperator, Mode
    from dips_amd.comm import Comm
    W, H, n = 448, 120, 41
    comm = Comm.rccl(Comm.unique_id(), 1, 0, 0)
    assert (comm.nranks, comm.rank) == (1, 0) and "rccl" in repr(comm)
    fmt = _fmt(fmt_name)
    c = int(fmt)
    op = DiffSeriesOperator(fmt, Mode(mode), TAU)
    try:
        fr = torch.empty((n,) + _shape(c, H, W), dtype=torch.uint8, device="cuda")
        op.synth_device(fr, W, H, SEED, 3)
        ref = torch.empty(_shape(c, H, W), dtype=torch.uint8, device="cuda")
        op.synth_device(ref.unsqueeze(0), W, H, SEED, 90)
        for r in (None, ref):
            one = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
            op.run_device(fr, one, ref=r)
            loc = torch.zeros_like(one)
            full = torch.full_like(one, -1)
            op.run_sharded(comm, fr, n, loc, full, ref=r)
            torch.cuda.synchronize()
            assert torch.equal(full, one) and torch.equal(loc, one)
            # series_all may begin at series_local (rank 0)
            alias = torch.zeros_like(one)
            op.run_sharded(comm, fr, n, alias, alias, ref=r)
            torch.cuda.synchronize()
            assert torch.equal(alias, one)
            # host pointers
            loc_h, full_h = op.sharded(comm, fr.cpu().numpy(), n, ref=r.cpu().numpy() if r is not None else None)
            assert np.array_equal(full_h.as_array(), one.cpu().numpy().view(np.uint64))
        # the broadcast on its own
        out = torch.zeros_like(ref)
        op.shard_broadcast_device(comm, ref, out)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    finally:
        op.close()
        comm.close()


def test_rccl_all_in_process():
    """dips_comm_create_all (ncclCommInitAll): every rank of one process, at
    one device here; the sharded call over it equals dips_diff_series."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from dips_amd.comm import Comm
    comms = Comm.rccl_all([0])
    assert len(comms) == 1 and (comms[0].nranks, comms[0].rank) == (1, 0) and "rccl" in repr(comms[0])
    W, H, n = 320, 96, 19
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, TAU)
    try:
        fr = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(fr, W, H, SEED, 0)
        one = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        op.run_device(fr, one)
        full = torch.zeros_like(one)
        op.run_sharded(comms[0], fr, n, full, full)
        torch.cuda.synchronize()
        assert torch.equal(full, one)
    finally:
        op.close()
        for c in comms:
            c.close()


def test_rccl_world1_bench_shape():
    """4K RGB8 'per-frame' at the bench's part-major size (600 frames) over
    RCCL at world size 1 equals dips_diff_series."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    from dips_amd.comm import Comm
    W, H, n = 3840, 2160, 600
    comm = Comm.rccl(Comm.unique_id(), 1, 0, 0)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, TAU)
    try:
        fr = torch.empty((n, H, W, 3), dtype=torch.uint8, device="cuda")
        op.synth_device(fr, W, H, SEED, 0)
        one = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
        op.run_device(fr, one)
        full = torch.zeros_like(one)
        op.run_sharded(comm, fr, n, full, full)
        torch.cuda.synchronize()
        assert torch.equal(full, one)
        p = op.shard_plan(comm, W, H, n)
        assert p["waves"] == p["waves_uncapped"]  # no halo at one rank: no reserve
    finally:
        op.close()
        comm.close()


# -- errors --------------------------------------------------------------------
def test_sharded_argument_errors():
    import torch
    from dips_amd import DiffSeriesOperator, DipsError, Mode, PixelFormat
    from dips_amd import _lib
    from dips_amd.comm import Comm
    comms = Comm.loopback(2, 0)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, TAU)
    try:
        W, H = 64, 32
        fr = torch.zeros((5, H, W, 3), dtype=torch.uint8, device="cuda")
        loc = torch.zeros((5, 4), dtype=torch.int64, device="cuda")
        full = torch.zeros((10, 4), dtype=torch.int64, device="cuda")
        # rank 0 of 2 over 11 frames owns 5; 10 frames would give it 5 too, 12 -> 6
        with pytest.raises(DipsError) as ei:
            op.run_sharded(comms[0], fr, 12, loc, torch.zeros((12, 4), dtype=torch.int64, device="cuda"))
        assert ei.value.status == _lib.DIPS_ERR_INVALID and "owns 6 frames" in str(ei.value)
        with pytest.raises(DipsError) as ei:  # fewer frames than ranks
            op.run_sharded(comms[0], fr[:0].view(0, H, W, 3), 1, loc[:0], full[:1])
        assert "at least one frame" in str(ei.value)
        with pytest.raises(ValueError):  # rank 0 without series_all
            op.run_sharded(comms[0], fr, 10, loc, None)
        lib = _lib.load()
        assert lib.dips_diff_series_sharded(op._dev.ptr, None, W, H, fr.data_ptr(), 5, 10, None, 0,
                                            loc.data_ptr(), full.data_ptr()) == _lib.DIPS_ERR_INVALID
        assert b"null communicator" in lib.dips_last_error(op._dev.ptr)
        assert lib.dips_diff_series_sharded(op._dev.ptr, comms[0].ptr, W, H, fr.data_ptr(), 5, 10, None, 2,
                                            loc.data_ptr(), full.data_ptr()) == _lib.DIPS_ERR_INVALID
        assert b"shard_flags" in lib.dips_last_error(op._dev.ptr)
    finally:
        op.close()
        for c in comms:
            c.close()


# -- the dips-compat ComputeState over frame ranges ----------
def _compat_loopback(world, n_total, w, h, props, device_ptrs):
    import torch
    from dips_amd import ComputeState
    from dips_amd.comm import Comm, shard_range
    frames = np.random.default_rng(world * 100 + n_total).integers(0, 256, (n_total, h, w, 4), dtype=np.uint8)
    comms = Comm.loopback(world, 0)
    states = [ComputeState(*props) for _ in range(world)]
    outs, errors = [None] * world, []
    try:
        ranges = [shard_range(n_total, world, r) for r in range(world)]
        if device_ptrs:
            dev_in = [torch.from_numpy(frames[s:e].copy()).cuda() for s, e in ranges]
            dev_out = [torch.empty_like(t) for t in dev_in]
            torch.cuda.synchronize()

        def rank(r):
            try:
                s, e = ranges[r]
                if device_ptrs:
                    states[r].frame_callback_batch_sharded_device(comms[r], dev_in[r], dev_out[r], n_total)
                else:
                    outs[r] = states[r].frame_callback_batch_sharded(comms[r], w, h, frames[s:e], n_total)
            except Exception as ex:  # reported below
                errors.append((r, repr(ex)))

        threads = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=180)
        assert not any(t.is_alive() for t in threads) and not errors, errors
        if device_ptrs:
            torch.cuda.synchronize()
            outs = [o.cpu().numpy() for o in dev_out]
        return frames, np.concatenate(outs)
    finally:
        for c in states:
            c.close()
        for c in comms:
            c.close()


@pytest.mark.parametrize("world,n_total", [(2, 19), (3, 31)])
@pytest.mark.parametrize("window", [1, 3])
@pytest.mark.parametrize("device_ptrs", [False, True])
def test_compat_sharded_equals_one_compute_state(world, n_total, window, device_ptrs):
    """dips_frame_callback_batch_sharded over loopback ranks (fresh
    ComputeStates) gives every frame the output one ComputeState over the
    whole clip gives it, which the oracle's frame_callback pins."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter
    w, h = 48, 32
    props = (True, window, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    frames, got = _compat_loopback(world, n_total, w, h, props, device_ptrs)
    one = ComputeState(*props)
    try:
        want = one.frame_callback_batch(w, h, frames)
    finally:
        one.close()
    assert np.array_equal(got, want)
    cs = oracle.ComputeState(True, window, 5.0, 0, 0)
    ref = np.stack([oracle.frame_callback(w, h, f, cs) for f in frames])
    assert np.array_equal(got, ref)


def test_compat_sharded_layout_refused_everywhere():
    """A layout where a rank would start before frame 7 is refused on every
    rank with the same message (no rank is left in a collective)."""
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, DipsError
    from dips_amd.comm import Comm
    comms = Comm.loopback(2, 0)
    states = [ComputeState(False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_) for _ in range(2)]
    try:
        fr = np.zeros((6, 16, 16, 4), dtype=np.uint8)
        for r in range(2):
            with pytest.raises(DipsError) as ei:
                states[r].frame_callback_batch_sharded(comms[r], 16, 16, fr, 12)
            assert "< 7" in str(ei.value)
    finally:
        for c in states:
            c.close()
        for c in comms:
            c.close()
