"""Randomized call-sequence parity of the dips-compat ComputeState
(dips/src/gpu/mod.rs:170-397, bind_groups.rs:407-427, lib.rs:233-246)
against the oracle's ComputeState: one fixed-seed sequence of ~300 random
operations per case, every output compared.

Host-pointer handle: add_texture, dispatch, frame_callback,
frame_callback_batch (host), start_texture, resume, dips_set_stream to
another stream or back.  Its device-pointer twin (its own ComputeState, see
ComputeState.frame_callback_batch_device) runs beside it on its own oracle:
frame_callback_batch_device, resume_device, start_texture_device, each on a
randomly chosen torch stream.  Cases: window 1 and 3, the deferred upload
on and off, an odd frame size and one cut into many ragged stripes.

This is the interleaving surface where round 2's raw-slot bug lived (a batch
right after an add_texture with no dispatch)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

N_OPS = 300


def _frame(rng, w, h, prev):
    """A random RGBA8 frame; now and then a repeat of the previous one or a
    small change of it (equal intensities, ties in the median)."""
    r = rng.random()
    if prev is not None and r < 0.15:
        return prev.copy()
    if prev is not None and r < 0.35:
        f = prev.copy()
        ys, xs = rng.integers(0, h, 20), rng.integers(0, w, 20)
        f[ys, xs] = rng.integers(0, 256, (20, 4), dtype=np.uint8)
        return f
    return rng.integers(0, 256, (h, w, 4), dtype=np.uint8)


@pytest.mark.parametrize("size", [(37, 23), (131, 61)])
@pytest.mark.parametrize("crosscheck", [False, True])
@pytest.mark.parametrize("window", [1, 3])
def test_random_call_sequences_match_oracle(window, crosscheck, size):
    import torch
    from dips_amd import ChromaFilter, ComputeState, DiPsFilter, frame_callback
    w, h = size
    # ragged row stripes for the per-frame paths: 2 per frame at 37x23, 5 at
    # 131x61 (host_stream.h piece_bytes); DIPS_FLAG_CROSSCHECK: no deferral,
    # no zero-copy stripes
    seed = 1000 * window + 10 * int(crosscheck) + w
    rng = np.random.default_rng(seed)
    props = (True, window, 3.0, 0, 2)  # colorized, sigmoid, green chroma
    gpu = ComputeState(props[0], window, props[2], DiPsFilter(props[3]), ChromaFilter(props[4]),
                       crosscheck=crosscheck)
    ora = oracle.ComputeState(*props)
    ora_dev = oracle.ComputeState(*props)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    lib, hd = gpu._hd._lib, gpu._hd
    prev = None
    log = []
    counts = {}
    try:
        for i in range(N_OPS):
            op = rng.choice(["add", "dispatch", "callback", "batch", "start", "resume", "stream",
                             "dev_batch", "dev_resume", "dev_start"],
                            p=[0.22, 0.20, 0.16, 0.10, 0.04, 0.04, 0.06, 0.12, 0.03, 0.03])
            counts[op] = counts.get(op, 0) + 1
            log.append(op)
            where = (i, op, log[-6:])
            if op == "add":
                prev = _frame(rng, w, h, prev)
                gpu.add_texture(w, h, prev)
                ora.add_texture(w, h, prev)
            elif op == "dispatch":
                a, b = gpu.dispatch(), ora.dispatch()
                assert (a is None) == (b is None), where
                if b is not None:
                    assert np.array_equal(a, b), (where, np.argwhere(a != b)[:4])
            elif op == "callback":
                prev = _frame(rng, w, h, prev)
                a = frame_callback(w, h, prev, gpu)
                b = oracle.frame_callback(w, h, prev, ora)
                assert np.array_equal(a, b), (where, np.argwhere(a != b)[:4])
            elif op == "batch":
                fr = []
                for _ in range(int(rng.integers(1, 7))):
                    prev = _frame(rng, w, h, prev)
                    fr.append(prev)
                fr = np.stack(fr)
                a = gpu.frame_callback_batch(w, h, fr)
                b = np.stack([oracle.frame_callback(w, h, f, ora) for f in fr])
                assert np.array_equal(a, b), (where, np.argwhere(a != b)[:4])
            elif op == "start":
                a, b = gpu.start_texture(), ora.start_texture()
                assert (a is None) == (b is None), where
                if b is not None:
                    assert np.array_equal(a, b), where
            elif op == "resume":
                start = ora.start_texture()
                if start is None:
                    start = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
                halo = np.stack([_frame(rng, w, h, prev) for _ in range(3)])
                t0 = int(rng.integers(7, 80))
                gpu.resume(w, h, start, halo, t0)
                ora.resume(w, h, start, halo, t0)
                prev = halo[-1]
            elif op == "stream":
                k = int(rng.integers(0, 3))
                s = None if k == 2 else ctypes.c_void_p(int(streams[k].cuda_stream))
                hd.check(lib.dips_set_stream(hd.ptr, s))
            elif op == "dev_batch":
                n = int(rng.integers(1, 6))
                fr = np.stack([_frame(rng, w, h, None) for _ in range(n)])
                s = streams[int(rng.integers(0, 2))]
                dev = torch.from_numpy(fr).cuda()
                out = torch.empty_like(dev)
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    gpu.frame_callback_batch_device(dev, out)
                s.synchronize()
                b = np.stack([oracle.frame_callback(w, h, f, ora_dev) for f in fr])
                assert np.array_equal(out.cpu().numpy(), b), where
            elif op == "dev_resume":
                start = ora_dev.start_texture()
                if start is None:
                    start = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
                halo = rng.integers(0, 256, (3, h, w, 4), dtype=np.uint8)
                t0 = int(rng.integers(7, 80))
                s = streams[int(rng.integers(0, 2))]
                sd, hdv = torch.from_numpy(start).cuda(), torch.from_numpy(halo).cuda()
                torch.cuda.synchronize()
                gpu.resume_device(sd, hdv, t0, stream=s.cuda_stream)
                s.synchronize()
                ora_dev.resume(w, h, start, halo, t0)
            elif op == "dev_start":
                out = torch.zeros((h, w, 4), dtype=torch.uint8, device="cuda")
                torch.cuda.synchronize()
                s = streams[int(rng.integers(0, 2))]
                ok = gpu.start_texture_device(out, stream=s.cuda_stream)
                s.synchronize()
                b = ora_dev.start_texture()
                assert ok == (b is not None), where
                if b is not None:
                    assert np.array_equal(out.cpu().numpy(), b), where
        # drain: a final dispatch / start texture on both handles agree
        a, b = gpu.dispatch(), ora.dispatch()
        assert (a is None) == (b is None)
        if b is not None:
            assert np.array_equal(a, b)
    finally:
        hd.check(lib.dips_set_stream(hd.ptr, None))  # never left on a test stream
        gpu.close()
        torch.cuda.synchronize()
    # the sequence exercised every operation
    assert all(counts.get(k, 0) > 0 for k in ("add", "dispatch", "callback", "batch", "start", "resume",
                                               "stream", "dev_batch", "dev_resume", "dev_start")), counts
