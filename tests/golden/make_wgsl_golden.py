"""Generate the wgsl_* golden fixtures (TEST INFRASTRUCTURE).

Unlike make_golden.py (fixtures from the numpy restatement), these outputs
come from the reference's own shader files, executed by oracle/wgsl_exec.py
(oracle/wgsl_ref.py restates only the Rust host side: the frame ring, the
start-texture pass, the uniform index, the dips_alt texture splice and run
loop).  Each fixture is accepted only where the C oracle agrees bit for bit,
and the manifest records the sha256 of every shader file and the pins under
which it was executed.  Needs the reference checkout (DIPS_REFERENCE_ROOT,
default /root/reference); the committed .npz files are what the tests read.

Run: python tests/golden/make_wgsl_golden.py   (writes wgsl_*.npz + wgsl_manifest.json here)
"""
import dataclasses
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle  # noqa: E402
from oracle import wgsl_ref  # noqa: E402
from oracle.wgsl_exec import PINS  # noqa: E402

DISPATCH = -1  # in an op sequence: dispatch(); k >= 0: add_texture(frames[k])


def content(kind, shape, rng):
    """RGBA8 frames [n, h, w, 4] of one kind of content."""
    n, h, w = shape
    if kind == "random":
        return rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
    if kind == "ties":  # max + min odd at every pixel: I * 255 lands on k + 0.5
        f = rng.integers(0, 256, (n, h, w, 4), dtype=np.uint8)
        mx, mn = f[..., :3].max(-1).astype(int), f[..., :3].min(-1).astype(int)
        even = (mx + mn) % 2 == 0
        am = f[..., :3].argmax(-1)
        fix = np.where(mx < 255, 1, -1)
        for c in range(3):
            sel = even & (am == c)
            f[..., c] = np.where(sel, f[..., c] + np.where(sel, fix, 0), f[..., c]).astype(np.uint8)
        return f
    if kind == "extreme":  # 0 / 255 channels: |diff| = 1 -> the inverse sigmoid's log(0), 1/0
        return (rng.integers(0, 2, (n, h, w, 4)) * 255).astype(np.uint8)
    if kind == "gray":
        g = rng.integers(0, 256, (n, h, w, 1), dtype=np.uint8)
        return np.concatenate([g, g, g, np.full_like(g, 255)], axis=-1)
    if kind == "smooth":  # small frame-to-frame changes around a gradient
        y, x = np.mgrid[0:h, 0:w]
        base = (x * 7 + y * 11) % 256
        f = np.empty((n, h, w, 4), np.uint8)
        for t in range(n):
            noise = rng.integers(-3, 4, (h, w, 4))
            f[t] = np.clip(base[..., None] + np.array([0, 40, 80, 0]) + noise + t, 0, 255)
        return f
    raise ValueError(kind)


def mixed_frames(n, h, w, rng, kinds):
    f = np.concatenate([content(kinds[t % len(kinds)], (1, h, w), rng) for t in range(n)])
    if n > 5:
        f[5] = f[4]  # an exact repeat
    return f


# (colorize, window, sensitivity, filter, chroma), (w, h), frames, kinds, op sequence
CS_CASES = [
    ((False, 1, 5.0, 255, 0), (24, 16), 8, ["random"], None),
    ((True, 1, 5.0, 0, 0), (19, 13), 8, ["ties", "random"], None),
    ((True, 1, 5.0, 1, 0), (19, 13), 8, ["extreme", "random"], None),
    ((False, 1, 3.0, 1, 2), (33, 17), 8, ["smooth"], None),
    ((True, 1, 5.0, 0, 1), (16, 16), 8, ["random", "gray"], None),
    ((False, 1, 5.0, 0, 3), (17, 1), 8, ["random"], None),
    ((True, 1, -3.0, 0, 0), (1, 18), 8, ["ties"], None),
    ((True, 1, 200.0, 1, 0), (20, 9), 8, ["smooth", "extreme"], None),
    ((False, 1, 1e-30, 1, 0), (20, 9), 8, ["random"], None),
    ((True, 1, 0.0, 0, 2), (20, 9), 8, ["random"], None),
    ((True, 2, 5.0, 255, 0), (21, 14), 8, ["random", "ties"], None),
    ((False, 3, 5.0, 0, 0), (21, 14), 7, ["smooth"], None),
    ((True, 4, 2.0, 1, 1), (18, 18), 7, ["random"], None),
    ((False, 5, 5.0, 255, 3), (18, 11), 7, ["ties", "gray"], None),
    ((True, 6, 5.0, 0, 0), (17, 12), 7, ["random"], None),
    ((True, 7, 0.7, 1, 0), (17, 12), 7, ["extreme", "smooth"], None),
    ((False, 11, 5.0, 0, 0), (19, 13), 6, ["random"], None),
    # repeated dispatches and add_texture without a dispatch
    ((True, 1, 5.0, 0, 0), (22, 10), 9, ["random", "ties"],
     [0, DISPATCH, 1, 2, DISPATCH, 3, DISPATCH, DISPATCH, 4, 5, DISPATCH, 6, DISPATCH, DISPATCH, 7, 8, DISPATCH]),
    ((False, 3, 5.0, 1, 0), (22, 10), 8, ["smooth"],
     [0, 1, 2, 3, DISPATCH, DISPATCH, 4, DISPATCH, 5, 6, DISPATCH, 7, DISPATCH, DISPATCH]),
]

# added after the first set (generated after ALT_CASES, so that the earlier
# fixtures keep their random frames): the windows 8-10, a window wider than
# the frame, and a long op sequence that turns the ring over several times
CS_CASES_2 = [
    ((True, 8, 5.0, 0, 0), (16, 12), 6, ["random", "ties"], None),
    ((False, 9, 5.0, 1, 1), (15, 11), 6, ["smooth"], None),
    ((True, 10, 2.0, 255, 2), (14, 13), 6, ["random"], None),
    ((True, 9, 5.0, 0, 3), (5, 4), 6, ["extreme", "random"], None),
    ((True, 1, 5.0, 1, 0), (13, 7), 16, ["random", "smooth", "ties"],
     [0, 1, DISPATCH, 2, 3, 4, DISPATCH, DISPATCH, 5, DISPATCH, 6, 7, 8, 9, DISPATCH, 10, DISPATCH, 11,
      DISPATCH, 12, 13, 14, 15, DISPATCH, DISPATCH]),
]

# (num_textures, colorize, window, scalar, filter, chroma), (w, h), frames, kinds, refresh markers
ALT_CASES = [
    ((2, True, 1, 5.0, 0, 0), (24, 14), 10, ["random"], [5]),
    ((2, False, 1, 3.0, 1, 2), (19, 13), 10, ["ties", "random"], []),
    ((2, True, 3, 5.0, 1, 0), (17, 12), 10, ["extreme", "random"], [4, 7]),
    ((3, True, 1, 5.0, 0, 1), (33, 17), 9, ["smooth"], [5]),
    ((2, False, 5, 1.0, 0, 3), (18, 11), 8, ["random", "gray"], []),
    ((1, True, 1, 10.0, 0, 0), (16, 16), 8, ["random"], [3]),
    ((5, True, 3, 5.0, 0, 0), (18, 9), 9, ["ties"], [6]),
    ((4, False, 7, 0.7, 1, 0), (17, 10), 8, ["smooth", "random"], []),
    ((16, True, 1, 5.0, 1, 2), (20, 9), 20, ["random", "extreme"], [17]),
    ((2, True, 2, 5.0, 0, 0), (1, 18), 8, ["random"], [5]),
]


# added after the first sets, generated last: the dips_alt windows 4, 6, 9
# and 11, a frame narrower than the window, and a long loop with several
# refresh markers
ALT_CASES_2 = [
    ((2, True, 4, 5.0, 0, 0), (15, 11), 8, ["random", "ties"], [5]),
    ((3, False, 6, 2.0, 1, 1), (14, 10), 8, ["smooth"], []),
    ((2, True, 9, 5.0, 0, 2), (13, 9), 7, ["random"], [4]),
    ((2, True, 11, 5.0, 1, 0), (6, 5), 7, ["extreme", "random"], []),
    ((4, True, 1, 5.0, 0, 3), (17, 8), 24, ["random", "smooth", "gray"], [6, 11, 12, 19]),
]


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    if os.path.exists(path):
        with np.load(path, allow_pickle=False) as z:
            if set(z.files) == set(arrays) and all(np.array_equal(z[k], v) for k, v in arrays.items()):
                return
    np.savez_compressed(path, **arrays)


def run_cs(cs, frames, ops, w, h):
    outs, some = [], []
    for op in ops:
        if op == DISPATCH:
            o = cs.dispatch()
            some.append(o is not None)
            if o is not None:
                outs.append(o)
        else:
            cs.add_texture(w, h, frames[op])
    return np.stack(outs) if outs else np.zeros((0, h, w, 4), np.uint8), np.array(some)


def default_ops(n):
    ops = []
    for k in range(n):
        ops += [k, DISPATCH]
    return ops


def main():
    if not wgsl_ref.available():
        sys.exit(f"reference shaders not found under {wgsl_ref.REF_ROOT}")
    manifest = {
        "generator": "tests/golden/make_wgsl_golden.py: the reference's shader files executed by "
                     "oracle/wgsl_exec.py, host side restated in oracle/wgsl_ref.py; each fixture "
                     "accepted only where the C oracle agrees bit for bit",
        "shaders": {p: wgsl_ref.shader_sha256(p) for p in
                    (wgsl_ref.DIPS_SHADER, wgsl_ref.DIPS_PRE_SHADER, wgsl_ref.ALT_SHADER)},
        "pins": dataclasses.asdict(PINS),
        "compute_state": [],
        "alt": [],
    }
    rng = np.random.default_rng(20261018)

    def cs_fixture(idx, params, w, h, n, kinds, ops):
        t0 = time.time()
        frames = mixed_frames(n, h, w, rng, kinds)
        ops = ops or default_ops(n)
        outs, some = run_cs(wgsl_ref.ComputeState(*params), frames, ops, w, h)
        o_c, some_c = run_cs(oracle.ComputeState(*params), frames, ops, w, h)
        assert np.array_equal(some, some_c) and np.array_equal(outs, o_c), ("C oracle disagrees", params)
        name = f"wgsl_cs_{idx:02d}.npz"
        _save(name, frames=frames, ops=np.array(ops, np.int32), outputs=outs, some=some)
        manifest["compute_state"].append({"file": name, "params": list(params), "width": w, "height": h,
                                          "content": kinds})
        print(f"{name} {params} {w}x{h} {time.time() - t0:.1f}s", flush=True)

    for idx, (params, (w, h), n, kinds, ops) in enumerate(CS_CASES):
        cs_fixture(idx, params, w, h, n, kinds, ops)

    def alt_fixture(idx, params, w, h, n, kinds, markers):
        t0 = time.time()
        frames = mixed_frames(n, h, w, rng, kinds)
        n_tex, col, win, k, filt, chroma = params
        outs = wgsl_ref.AltCompute(n_tex, w, h, col, win, k, filt, chroma).run(frames, markers)
        o_c = oracle.AltCompute(n_tex, w, h, col, win, k, filt, chroma).run(frames, markers)
        assert np.array_equal(outs, o_c), ("C oracle disagrees", params)
        name = f"wgsl_alt_{idx:02d}.npz"
        _save(name, frames=frames, outputs=outs)
        manifest["alt"].append({"file": name, "num_textures": n_tex, "colorize": col, "window": win,
                                "scalar": k, "filter": filt, "chroma": chroma, "markers": markers,
                                "content": kinds})
        print(f"{name} {params} {w}x{h} {time.time() - t0:.1f}s", flush=True)

    for idx, (params, (w, h), n, kinds, markers) in enumerate(ALT_CASES):
        alt_fixture(idx, params, w, h, n, kinds, markers)
    for idx, (params, (w, h), n, kinds, ops) in enumerate(CS_CASES_2):
        cs_fixture(len(CS_CASES) + idx, params, w, h, n, kinds, ops)
    for idx, (params, (w, h), n, kinds, markers) in enumerate(ALT_CASES_2):
        alt_fixture(len(ALT_CASES) + idx, params, w, h, n, kinds, markers)
    with open(os.path.join(HERE, "wgsl_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"wrote {len(manifest['compute_state'])} ComputeState + {len(manifest['alt'])} dips_alt fixtures")


if __name__ == "__main__":
    main()
