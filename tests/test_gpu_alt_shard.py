"""The native frame-range sharding of the dips_alt run loop
(include/dips_hip.h dips_alt_run_sharded, alt_abi.hip) through the C ABI, on
the one GPU of the box, ranks as loopback threads:

* every rank's outputs equal one run_dips_on_file loop over every frame
  (dips_alt/src/lib.rs:588-683; DiPsRunner, itself pinned to the oracle in
  test_gpu_alt.py) and the oracle's loop (oracle.AltCompute.run), for world
  sizes 2, 3 and 8, refresh markers on and across the range edges, the batch
  kernel (N = 2, W = 1) and the per-frame kernel (N = 3, W = 3), host and
  device pointers;
* the splits the replay must get right: a rank starting before frame
  num_textures after a snapshot (zero frames before its halo), ranks with no
  frame, a snapshot many frames before a rank's first frame;
* the loop state after the call is the single loop's: the last rank carries
  on with more frames through the ordinary run;
* argument and state errors return on the rank that has them.

The reference is single-device; the sharding is SURVEY.md s8e's."""
import threading

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _frames(w, h, n, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    if n > 5:
        f[5] = f[4]  # a still frame: zero differences
    return f


def _props(window=1, filt=0, colorize=True, chroma=0):
    from dips_amd.alt import ChromaFilter, DiPsProperties
    return DiPsProperties(colorize=colorize, window_size=window, sigmoid_horizontal_scalar=5.0,
                          filter_type=filt, chroma_filter=ChromaFilter(chroma))


def _one_loop(frames, props, markers, n_tex):
    from dips_amd.alt import DiPsRunner
    r = DiPsRunner(frames.shape[1], frames.shape[2], props, markers, num_textures=n_tex)
    try:
        return r(frames)
    finally:
        r.close()


def _sharded(world, frames, props, markers, n_tex, device_ptrs, keep_last=False, crosscheck=False):
    """dips_alt_run_sharded on `world` loopback ranks, one thread each;
    returns the concatenated outputs (and the last rank's runner if asked)."""
    import torch
    from dips_amd.alt import DiPsRunner
    from dips_amd.comm import Comm, shard_range
    n, h, w = frames.shape[:3]
    comms = Comm.loopback(world, 0)
    runners = [DiPsRunner(h, w, props, markers, num_textures=n_tex, crosscheck=crosscheck) for _ in range(world)]
    outs, errs = [None] * world, [None] * world

    def rank(r):
        try:
            s, e = shard_range(n, world, r)
            if device_ptrs:
                dev = torch.from_numpy(frames[s:e].copy()).cuda()
                out = torch.empty_like(dev)
                runners[r].run_sharded_device(comms[r], dev, out, n)
                outs[r] = out.cpu().numpy()
            else:
                outs[r] = runners[r].run_sharded(comms[r], frames[s:e], n)
        except Exception as ex:  # reported below, on the test's thread
            errs[r] = ex

    if device_ptrs:
        torch.cuda.synchronize()
    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    try:
        assert not any(t.is_alive() for t in th), "a rank did not return"
        assert errs == [None] * world, errs
        got = np.concatenate(outs) if n else np.empty((0, h, w, 4), dtype=np.uint8)
        if keep_last:
            last = runners.pop()
            return got, last
        return got
    finally:
        for r in runners:
            r.close()
        for c in comms:
            c.close()


CASES = [
    # world, n, n_tex, window, markers
    (2, 48, 2, 1, [5, 6, 30]),
    (3, 48, 2, 1, [16, 17, 32, 40]),     # resets on and just after the range edges 16, 32
    (8, 20, 2, 1, []),                   # one snapshot (frame 2), far before most ranks
    (8, 10, 4, 1, []),                   # rank 3 starts at 3 < N = 4 after the snapshot at 2
    (8, 5, 2, 1, [3]),                   # ranks with no frame
    (3, 30, 3, 3, [4, 11, 12, 25]),      # per-frame kernel, spatial window
]


@pytest.mark.parametrize("device_ptrs", [False, True])
@pytest.mark.parametrize("world,n,n_tex,window,markers", CASES)
def test_alt_sharded_equals_one_loop(world, n, n_tex, window, markers, device_ptrs):
    w, h = (40, 24) if window == 1 else (37, 21)
    frames = _frames(w, h, n, 300 + world + n)
    props = _props(window)
    want = _one_loop(frames, props, markers, n_tex)
    got = _sharded(world, frames, props, markers, n_tex, device_ptrs)
    assert got.shape == want.shape
    bad = np.argwhere(np.any(got != want, axis=(1, 2, 3)))
    assert bad.size == 0, f"frames differing from the single loop: {bad.ravel()[:8]}"


@pytest.mark.parametrize("device_ptrs", [False, True])
def test_alt_sharded_crosscheck_kernels(device_ptrs):
    """DIPS_FLAG_CROSSCHECK (the arithmetic epilogue instead of the table,
    host frames through the pinned buffer) under the sharded call."""
    w, h, n, markers = 40, 24, 33, [9, 10, 21]
    frames = _frames(w, h, n, 123)
    props = _props(1, 1, True, 3)
    want = _one_loop(frames, props, markers, 2)
    got = _sharded(3, frames, props, markers, 2, device_ptrs, crosscheck=True)
    assert np.array_equal(got, want)


def test_alt_sharded_no_frames():
    """n_total = 0: every rank owns nothing and returns at once."""
    frames = np.zeros((0, 8, 16, 4), dtype=np.uint8)
    got = _sharded(3, frames, _props(), [], 2, False)
    assert got.shape == (0, 8, 16, 4)


@pytest.mark.parametrize("world", [2, 3])
def test_alt_sharded_matches_oracle(world):
    w, h, n, markers = 64, 32, 40, [7, 19, 20, 33]
    frames = _frames(w, h, n, 77 + world)
    got = _sharded(world, frames, _props(1, 1, False, 2), markers, 2, True)
    want = oracle.AltCompute(2, w, h, False, 1, 5.0, 1, 2).run(frames, markers)
    assert np.array_equal(got, want), np.argwhere(got != want)[:4]


def test_alt_sharded_loop_state_carries_on():
    """After the sharded call the last rank's runner holds the single loop's
    state: its next ordinary call continues that loop."""
    w, h, n, extra, markers = 40, 24, 36, 12, [13, 30, 41]
    frames = _frames(w, h, n + extra, 91)
    props = _props()
    want = _one_loop(frames, props, markers, 2)
    got, last = _sharded(3, frames[:n], props, markers, 2, False, keep_last=True)
    try:
        assert np.array_equal(got, want[:n])
        more = last(frames[n:])
        assert np.array_equal(more, want[n:])
    finally:
        last.close()


def test_alt_sharded_errors():
    from dips_amd import _lib
    from dips_amd.alt import DiPsRunner
    from dips_amd.comm import Comm
    w, h = 40, 24
    frames = _frames(w, h, 6, 5)
    (comm,) = Comm.loopback(1, 0)
    r = DiPsRunner(h, w, _props())
    try:
        with pytest.raises(_lib.DipsError) as e:
            r.run_sharded(comm, frames[:4], 6)  # owns all 6 frames
        assert e.value.status == _lib.DIPS_ERR_INVALID and "owns 6 frames, n_local is 4" in str(e.value)
        r(frames[:2])
        with pytest.raises(_lib.DipsError) as e:
            r.run_sharded(comm, frames, 6)  # not fresh
        assert e.value.status == _lib.DIPS_ERR_STATE and "fresh" in str(e.value)
    finally:
        r.close()
        comm.close()
    # one rank of a fresh runner: the same as the ordinary run
    (comm,) = Comm.loopback(1, 0)
    r = DiPsRunner(h, w, _props(), [3])
    try:
        got = r.run_sharded(comm, frames, 6)
    finally:
        r.close()
        comm.close()
    assert np.array_equal(got, _one_loop(frames, _props(), [3], 2))
