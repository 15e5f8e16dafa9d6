"""Generate the committed golden fixtures (TEST INFRASTRUCTURE).

The reference (Rust + WGSL through wgpu) cannot run in this image and ships
no fixtures, so the fixtures are produced by the
independent numpy restatement (oracle/np_restatement.py) and accepted only
where the C oracle (oracle/dips_oracle.c) agrees bit for bit.  They pin the
oracle against regressions; the pin against the reference's shader text is
make_wgsl_golden.py's (DESIGN.md "Oracle").

Run: python tests/golden/make_golden.py   (writes *.npz + manifest.json here)
"""
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import np_restatement as nr  # noqa: E402
from oracle import oracle  # noqa: E402


def _save(name, **arrays):
    """Write a fixture unless an identical one is already committed (keeps
    the bytes of existing fixtures stable across regenerations)."""
    path = os.path.join(HERE, name)
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as z:
            if set(z.files) == set(arrays) and all(np.array_equal(z[k], v) for k, v in arrays.items()):
                return
    np.savez_compressed(path, **arrays)


def boundary_pools(tau: float):
    """Pixel pairs (reference, current) whose f32 |dI| is one ulp below,
    exactly equal to and one ulp above f32(tau) (dips_shader.wgsl:64-82
    intensity; the series counts dI > tau, strictly).  Returns
    {chroma_kind: {cat: [(p, q), ...]}} with chroma_kind "none" (p, q are
    (max, min) byte pairs) or "channel" (p, q are bytes)."""
    F32 = np.float32
    t = F32(tau)
    cats = {"below": np.nextafter(t, F32(0)), "equal": t, "above": np.nextafter(t, F32(1))}
    U = nr.U_LUT
    out = {"channel": {}, "none": {}}
    a, b = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    d = np.abs((U[a] - U[b]).astype(F32))
    for k, v in cats.items():
        out["channel"][k] = [tuple(map(int, x)) for x in np.argwhere(d == v)]
    mx, mn = np.meshgrid(np.arange(256), np.arange(256), indexing="ij")
    keep = mx >= mn
    mx, mn = mx[keep], mn[keep]
    iv = ((U[mx] + U[mn]).astype(F32) / F32(2.0)).astype(F32)
    for k, v in cats.items():
        pairs = []
        for i in range(0, len(mx), 7):  # a deterministic subsample of references
            j = np.where(np.abs((iv - iv[i]).astype(F32)) == v)[0]
            pairs += [((int(mx[i]), int(mn[i])), (int(mx[x]), int(mn[x]))) for x in j[:3]]
            if len(pairs) >= 400:
                break
        out["none"][k] = pairs
    for kind in out:
        for k in cats:
            assert out[kind][k], (kind, k)
    return out


def boundary_frames(c: int, chroma: int, w: int, h: int, pools, rng) -> np.ndarray:
    """Three frames: frame 0 the references, frame 1 pixels whose |dI| to
    frame 0 is one ulp below / equal to / one ulp above tau (or random),
    frame 2 frame 1 with pixels swapped back to frame 0 in places."""
    shape = (3, h, w) if c == 1 else (3, h, w, c)
    f = rng.integers(0, 256, shape, dtype=np.uint8)
    kind = "none" if (chroma == 0 and c != 1) else "channel"
    cats = ["below", "equal", "above", "random"]
    for y in range(h):
        for x in range(w):
            cat = cats[rng.integers(0, 4)]
            if cat == "random":
                continue
            pool = pools[kind][cat]
            p, q = pool[rng.integers(0, len(pool))]
            if rng.integers(0, 2):
                p, q = q, p
            for t, v in ((0, p), (1, q)):
                if c == 1:
                    f[t, y, x] = v
                elif kind == "none":
                    hi, lo = v
                    px = [hi, lo, int(rng.integers(lo, hi + 1))]
                    rng.shuffle(px)
                    f[t, y, x, :3] = px
                else:
                    f[t, y, x, chroma - 1] = v
    swap = rng.integers(0, 2, (h, w)).astype(bool)
    f[2][swap] = f[0][swap]
    return f


def _series_case(manifest, idx, frames, c, mode, chroma, tau, ref, w, h, tag):
    out4, si, dmap = nr.series(frames, mode=mode, chroma=chroma, tau=tau, ref=ref)
    o4, si_c, dm_c = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, ref=ref, want_map=True)
    assert np.array_equal(out4, o4) and np.array_equal(dmap, dm_c)
    assert np.allclose(si, si_c, rtol=1e-12)
    name = f"series_{idx:02d}_c{c}_m{mode}_ch{chroma}_t{int(round(tau * 255))}{tag}.npz"
    arrays = dict(frames=frames, out4=out4, si=si_c, dmap=dmap)
    if ref is not None:
        arrays["ref"] = ref
    _save(name, **arrays)
    manifest["series"].append({"file": name, "channels": c, "mode": mode, "chroma": chroma,
                               "tau": tau, "width": w, "height": h, "frames": int(frames.shape[0]),
                               "ref": ref is not None, **({"tau_boundary": True} if tag else {})})
    return idx + 1


def main():
    manifest = {
        "generator": "tests/golden/make_golden.py (numpy restatement, cross-checked with the C oracle)",
        "pins": {
            "bounds_policy": "naga Restrict (Vulkan/DX12)",
            "unorm_load": "c / 255.0f (IEEE division)",
            "unorm_store": "rint(clamp(x,0,1)*255.0f), round half to even, NaN -> 0",
            "exp_log": "deterministic f32 algorithms of DESIGN.md",
            "spatial_filter_race": "filter reads the slot as it was before the dispatch",
        },
        "series": [],
        "compute_state": [],
    }
    rng = np.random.default_rng(20261015)
    cases = []
    for c, mode in itertools.product([1, 3, 4], [0, 1]):
        for chroma in ([0] if c == 1 else [0, 2]):
            for tau in (0.0, 8 / 255):
                cases.append((c, mode, chroma, tau))
    for idx, (c, mode, chroma, tau) in enumerate(cases):
        w, h = (64, 48) if idx % 2 == 0 else (37, 23)
        frames = nr.synth(c, w, h, 1 + idx, 0, 6)
        if idx % 3 == 0:  # mix in random frames and an exact repeat
            frames[2] = rng.integers(0, 256, frames[2].shape, dtype=np.uint8)
            frames[3] = frames[2]
        ref = rng.integers(0, 256, frames[0].shape, dtype=np.uint8) if idx % 4 == 1 else None
        out4, si, dmap = nr.series(frames, mode=mode, chroma=chroma, tau=tau, ref=ref)
        o4, si_c, dm_c = oracle.series(frames, mode=mode, chroma=chroma, tau=tau, ref=ref, want_map=True)
        assert np.array_equal(out4, o4) and np.array_equal(dmap, dm_c)
        assert np.allclose(si, si_c, rtol=1e-12)
        name = f"series_{idx:02d}_c{c}_m{mode}_ch{chroma}_t{int(round(tau * 255))}.npz"
        arrays = dict(frames=frames, out4=out4, si=si_c, dmap=dmap)
        if ref is not None:
            arrays["ref"] = ref
        _save(name, **arrays)
        manifest["series"].append({"file": name, "channels": c, "mode": mode, "chroma": chroma,
                                   "tau": tau, "width": w, "height": h, "frames": int(frames.shape[0]),
                                   "ref": ref is not None})
    cs_cases = [(False, 1, 5.0, 255, 0), (True, 1, 5.0, 0, 0), (False, 1, 3.0, 1, 2),
                (True, 3, 5.0, 255, 0), (False, 5, 2.0, 0, 1), (True, 2, 5.0, 1, 3)]
    for idx, params in enumerate(cs_cases):
        w, h = 24, 16
        frames = rng.integers(0, 256, (8, h, w, 4), dtype=np.uint8)
        frames[5] = frames[4]
        a = nr.ComputeState(*params)
        b = oracle.ComputeState(*params)
        outs = []
        for k in range(8):
            a.add_texture(w, h, frames[k])
            b.add_texture(w, h, frames[k])
            x, y = a.dispatch(), b.dispatch()
            assert (x is None) == (y is None)
            if x is not None:
                assert np.array_equal(x, y)
                outs.append(x)
        name = f"compute_state_{idx:02d}.npz"
        _save(name, frames=frames, outputs=np.stack(outs))
        manifest["compute_state"].append({"file": name, "params": list(params)})
    # dips_alt run loop (run_dips_on_file, dips_alt/src/lib.rs:588-683):
    # (num_textures, colorize, window, scalar, filter, chroma), refresh markers
    manifest["alt"] = []
    arng = np.random.default_rng(20261016)
    alt_cases = [(2, True, 1, 5.0, 0, 0), (2, False, 1, 3.0, 1, 2), (2, True, 4, 5.0, 1, 0),
                 (3, True, 1, 5.0, 0, 1), (2, False, 7, 0.7, 0, 3), (1, True, 2, 5.0, 0, 0)]
    for idx, (n_tex, col, win, k, filt, chroma) in enumerate(alt_cases):
        w, h = 24, 14
        frames = arng.integers(0, 256, (10, h, w, 4), dtype=np.uint8)
        frames[6] = frames[5]
        markers = [5] if idx % 2 == 0 else []
        a = nr.AltCompute(n_tex, w, h, col, win, k, filt, chroma).run(frames, markers)
        b = oracle.AltCompute(n_tex, w, h, col, win, k, filt, chroma).run(frames, markers)
        assert np.array_equal(a, b)
        name = f"alt_{idx:02d}.npz"
        _save(name, frames=frames, outputs=a)
        manifest["alt"].append({"file": name, "num_textures": n_tex, "colorize": col, "window": win,
                                "scalar": k, "filter": filt, "chroma": chroma, "markers": markers})
    # round 2: chroma Red / Blue (the series_v2 CH = 1, 3 instantiations) and
    # the strict dI > tau boundary (own generator, so the fixtures above keep
    # their bytes)
    rng2 = np.random.default_rng(20261016)
    idx = len(manifest["series"])
    for c, mode, chroma, tau in itertools.product([3, 4], [0, 1], [1, 3], [0.0, 8 / 255]):
        w, h = (64, 48) if idx % 2 == 0 else (37, 23)
        frames = nr.synth(c, w, h, 100 + idx, 0, 6)
        if idx % 3 == 0:
            frames[2] = rng2.integers(0, 256, frames[2].shape, dtype=np.uint8)
            frames[3] = frames[2]
        ref = rng2.integers(0, 256, frames[0].shape, dtype=np.uint8) if idx % 4 == 1 else None
        idx = _series_case(manifest, idx, frames, c, mode, chroma, tau, ref, w, h, "")
    pools = boundary_pools(8 / 255)
    for c in (1, 3, 4):
        for chroma in ([0] if c == 1 else [0, 1, 3]):
            for mode in (0, 1):
                w, h = (64, 48) if idx % 2 == 0 else (37, 23)
                frames = boundary_frames(c, chroma, w, h, pools, rng2)
                idx = _series_case(manifest, idx, frames, c, mode, chroma, 8 / 255, None, w, h, "_tauedge")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(manifest['series'])} series + {len(manifest['compute_state'])} ComputeState + "
          f"{len(manifest['alt'])} dips_alt fixtures")


if __name__ == "__main__":
    main()
