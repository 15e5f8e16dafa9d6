"""Independent numpy restatement of the DiPs path -- TEST INFRASTRUCTURE ONLY.

A second, independently written CPU statement of the same semantics as
``dips_oracle.c``, vectorised with float32 numpy arithmetic (IEEE, round to
nearest even, no FMA contraction).  It exists to cross-check the C oracle
(tests/test_oracle.py) and to generate the committed golden fixtures
(tests/golden/make_golden.py).  It is never shipped to or run by the product.

Reference semantics followed (RubenMovsesyan/DiPs):
  get_intensity            dips/src/gpu/shaders/dips_shader.wgsl:64-82
  spatial_median_filter    dips/src/gpu/shaders/dips_shader.wgsl:120-170
  compute_main             dips/src/gpu/shaders/dips_shader.wgsl:172-240
  pre_compute_main         dips/src/gpu/shaders/pre_compute_shader.wgsl:92-132
  ComputeState state       dips/src/gpu/mod.rs:170-216, bind_groups.rs:205-427
  callback passthrough     dips/src/lib.rs:233-246
"""
from __future__ import annotations

from typing import Optional

import numpy as np

F32 = np.float32
U_LUT = (np.arange(256, dtype=F32) / F32(255.0)).astype(F32)  # rgba8unorm load


def q(x: np.ndarray) -> np.ndarray:
    """rgba8unorm store: clamp, *255, round half even, NaN -> 0."""
    x = np.asarray(x, dtype=F32)
    with np.errstate(invalid="ignore"):
        y = np.where(x > F32(0.0), x, F32(0.0))
        y = np.where(y > F32(1.0), F32(1.0), y).astype(F32)
    return np.rint((y * F32(255.0)).astype(F32)).astype(np.uint8)


def _pow2i(n: np.ndarray) -> np.ndarray:
    return ((n.astype(np.int64) + 127) << 23).astype(np.uint32).view(F32)


def expf(x) -> np.ndarray:
    x = np.asarray(x, dtype=F32)
    with np.errstate(over="ignore", invalid="ignore"):
        xc = np.clip(x, F32(-103.97208404541016), F32(88.72283935546875)).astype(F32)
        kf = np.rint((xc * F32(1.44269502162933349609375)).astype(F32)).astype(F32)
        r = (xc - (kf * F32(0.693145751953125)).astype(F32)).astype(F32)
        r = (r - (kf * F32(1.428606765330187045e-06)).astype(F32)).astype(F32)
        p = np.full_like(r, F32(1.3888889225e-3))
        for c in (8.3333337680e-3, 4.1666667908e-2, 1.6666667163e-1, 0.5, 1.0, 1.0):
            p = ((p * r).astype(F32) + F32(c)).astype(F32)
        k = kf.astype(np.int32)
        k1 = np.trunc(k / 2).astype(np.int32)
        k2 = k - k1
        p = (p * _pow2i(k1)).astype(F32)
        p = (p * _pow2i(k2)).astype(F32)
    p = np.where(x > F32(88.72283935546875), F32(np.inf), p)
    p = np.where(x < F32(-103.97208404541016), F32(0.0), p)
    p = np.where(np.isnan(x), x, p)
    return p.astype(F32)


def logf(x) -> np.ndarray:
    x = np.asarray(x, dtype=F32)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        sub = (x > 0) & (x < F32(1.1754943508222875e-38))
        xs = np.where(sub, (x * F32(8388608.0)).astype(F32), x).astype(F32)
        bits = np.abs(xs).view(np.uint32)
        e = (bits >> 23).astype(np.int64) - 127 - np.where(sub, 23, 0)
        m = ((bits & np.uint32(0x007FFFFF)) | np.uint32(0x3F800000)).view(F32)
        big = m > F32(1.41421353816986083984375)
        m = np.where(big, (m * F32(0.5)).astype(F32), m).astype(F32)
        e = e + big
        f = (m - F32(1.0)).astype(F32)
        s = (f / (F32(2.0) + f).astype(F32)).astype(F32)
        z = (s * s).astype(F32)
        t = np.full_like(z, F32(1.1111111194e-1))
        for c in (1.4285714924e-1, 2.0000000298e-1, 3.3333334327e-1, 1.0):
            t = ((t * z).astype(F32) + F32(c)).astype(F32)
        lm = ((F32(2.0) * s).astype(F32) * t).astype(F32)
        ef = e.astype(F32)
        res = ((ef * F32(0.693145751953125)).astype(F32)
               + ((ef * F32(1.428606765330187045e-06)).astype(F32) + lm).astype(F32)).astype(F32)
    res = np.where(x == 0, F32(-np.inf), res)
    res = np.where(x == F32(np.inf), F32(np.inf), res)
    res = np.where(np.isnan(x) | (x < 0), F32(np.nan), res)
    return res.astype(F32)


def _rgb(frames: np.ndarray, gray: Optional[bool] = None):
    if gray is None:
        gray = frames.ndim == 3  # batched [N,H,W] gray8
    if gray:  # gray8: r = g = b
        return frames, frames, frames
    return frames[..., 0], frames[..., 1], frames[..., 2]


def intensity(frames: np.ndarray, chroma: int = 0, gray: Optional[bool] = None) -> np.ndarray:
    r, g, b = _rgb(frames, gray)
    fr, fg, fb = U_LUT[r], U_LUT[g], U_LUT[b]
    if chroma == 1:
        return fr
    if chroma == 2:
        return fg
    if chroma == 3:
        return fb
    cmax = np.maximum(np.maximum(fr, fg), fb)
    cmin = np.minimum(np.minimum(fr, fg), fb)
    return ((cmax + cmin).astype(F32) / F32(2.0)).astype(F32)


def jtwin(frames: np.ndarray, chroma: int = 0) -> np.ndarray:
    r, g, b = (a.astype(np.int64) for a in _rgb(frames))
    if chroma in (1, 2, 3):
        return 2 * (r, g, b)[chroma - 1]
    return np.maximum(np.maximum(r, g), b) + np.minimum(np.minimum(r, g), b)


def series(frames: np.ndarray, *, mode: int = 0, chroma: int = 0, tau: float = 0.0,
           ref: Optional[np.ndarray] = None):
    """Returns (out4 [N,4] uint64 = SAD, SJ, count, SI_fixed; si_f64 [N]; dmap)."""
    frames = np.asarray(frames, dtype=np.uint8)
    n = frames.shape[0]
    if mode == 0:
        refs = np.broadcast_to((frames[0] if ref is None else ref.reshape(frames.shape[1:]))[None],
                               frames.shape)
    else:
        first = frames[0] if ref is None else ref.reshape(frames.shape[1:])
        refs = np.concatenate([first[None], frames[:-1]], axis=0)
    d = np.abs(frames.astype(np.int16) - refs.astype(np.int16)).astype(np.uint8)
    axes = tuple(range(1, frames.ndim))
    sad = d.reshape(n, -1).astype(np.uint64).sum(axis=1)
    sj = np.abs(jtwin(frames, chroma) - jtwin(refs, chroma)).reshape(n, -1).sum(axis=1)
    dI = np.abs((intensity(frames, chroma) - intensity(refs, chroma)).astype(F32))
    sel = dI > F32(tau)
    cnt = sel.reshape(n, -1).sum(axis=1)
    fixed = np.where(sel, np.ldexp(dI.astype(np.float64), 32), 0.0).astype(np.uint64)
    sif = fixed.reshape(n, -1).sum(axis=1, dtype=np.uint64)
    si = np.array([np.add.reduce(np.where(s, x, F32(0)).astype(np.float64).ravel())
                   for s, x in zip(sel, dI)], dtype=np.float64) if n else np.zeros(0)
    del axes
    out4 = np.stack([sad, sj.astype(np.uint64), cnt.astype(np.uint64), sif], axis=1).astype(np.uint64)
    return out4, si, d


# --------------------------------------------------------------------------
# Synthetic generator
# --------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def synth(channels: int, width: int, height: int, seed: int, t0: int, n: int) -> np.ndarray:
    yy, xx, cc = np.meshgrid(np.arange(height, dtype=np.uint64), np.arange(width, dtype=np.uint64),
                             np.arange(channels, dtype=np.uint64), indexing="ij")
    idx = (yy * np.uint64(width) + xx) * np.uint64(channels) + cc
    base = (splitmix64(np.uint64(seed) ^ idx) & np.uint64(0xFF)).astype(np.int64)
    rad = max(height // 8, 1)
    out = np.empty((n, height, width, channels), dtype=np.uint8)
    for k in range(n):
        t = t0 + k
        fkey = splitmix64(np.array([(seed + t) & 0xFFFFFFFFFFFFFFFF], dtype=np.uint64))[0]
        cx = (width // 4 + 4 * t) % width
        cy = height // 2
        dx = xx.astype(np.int64) - cx
        dy = yy.astype(np.int64) - cy
        blob = np.where(dx * dx + dy * dy <= rad * rad, 64, 0)
        h = splitmix64(fkey ^ idx)
        noise = (((h >> np.uint64(32)) * np.uint64(9)) >> np.uint64(32)).astype(np.int64) - 4
        out[k] = np.clip(base + blob + noise, 0, 255).astype(np.uint8)
    return out[..., 0] if channels == 1 else out


# --------------------------------------------------------------------------
# dips-compat ComputeState
# --------------------------------------------------------------------------

def spatial(img: np.ndarray, window: int, chroma: int) -> np.ndarray:
    """spatial_median_filter on an RGBA image [H,W,4] -> filtered intensity [H,W]."""
    I = intensity(img[..., :3], chroma, gray=False)
    if window == 1:
        return I
    h, w = I.shape
    hw = window // 2
    size = window * window
    region = min(size, 120) + 1
    cols = []
    for i in range(-hw, hw):
        for j in range(-hw, hw):
            sh = np.zeros_like(I)
            ys, xs = np.arange(h) + j, np.arange(w) + i
            vy, vx = (ys >= 0) & (ys < h), (xs >= 0) & (xs < w)
            sub = I[np.clip(ys, 0, h - 1)][:, np.clip(xs, 0, w - 1)]
            sh = np.where(vy[:, None] & vx[None, :], sub, F32(0.0)).astype(F32)
            cols.append(sh)
    vals = np.stack(cols, axis=-1)
    zeros = np.zeros((h, w, region - vals.shape[-1]), dtype=F32)
    allv = np.sort(np.concatenate([vals, zeros], axis=-1), axis=-1)
    k = min(size // 2 + 1, 120)
    return allv[..., k].astype(F32)


def upper_median4(stack: np.ndarray) -> np.ndarray:
    return np.sort(stack, axis=-1)[..., 2]


def _sigmoid(x, k):
    return ((F32(1.0) / (F32(1.0) + expf((F32(-k) * x).astype(F32))).astype(F32)).astype(F32)
            - F32(0.5)).astype(F32)


def _inv_sigmoid(x, k):
    inner = ((F32(1.0) / (x + F32(0.5)).astype(F32)).astype(F32) - F32(1.0)).astype(F32)
    return ((-logf(inner)).astype(F32) / F32(k)).astype(F32)


def epilogue(diff: np.ndarray, filter_type: int, sensitivity: float, colorize: bool) -> np.ndarray:
    """dips_shader.wgsl:217-239: map, filter, *5, colorize; returns RGBA8."""
    with np.errstate(all="ignore"):
        d = (diff * F32(0.5)).astype(F32)
        if filter_type == 0:
            d = _sigmoid(d, sensitivity)
        elif filter_type == 1:
            d = _inv_sigmoid(d, sensitivity)
        d = (d * F32(5.0)).astype(F32)
        if colorize:
            neg = d < F32(0.0)
            s = np.where(neg, np.abs(d), d).astype(F32)
            chroma = s  # s * (1 - |2*0.5 - 1|) = s * 1
            m = (F32(0.5) - (chroma / F32(2.0)).astype(F32)).astype(F32)
            x = (chroma * F32(0.0)).astype(F32)
            hi = (chroma + m).astype(F32)
            lo = (F32(0.0) + m).astype(F32)
            xm = (x + m).astype(F32)
            r = np.where(neg, hi, lo)
            g = np.where(neg, xm, hi)
            b = np.where(neg, lo, xm)
        else:
            r = g = b = (F32(0.5) - d).astype(F32)
    out = np.empty(diff.shape + (4,), dtype=np.uint8)
    out[..., 0], out[..., 1], out[..., 2] = q(r), q(g), q(b)
    out[..., 3] = 255
    return out


class ComputeState:
    """numpy twin of ComputeState (dips/src/gpu/mod.rs:39-398)."""

    def __init__(self, colorize, spatial_window_size, sensitivity, filter_type, chroma_filter):
        self.colorize = bool(colorize)
        self.window = int(spatial_window_size)
        self.k = float(np.float32(sensitivity))
        self.filter = int(filter_type)
        self.chroma = int(chroma_filter)
        self.queue = []
        self.start = None
        self.slots = None
        self.ring = 0
        self.uniform = 0

    def add_texture(self, width, height, frame):
        frame = np.asarray(frame, dtype=np.uint8).reshape(height, width, 4).copy()
        self.queue.append(frame)
        if len(self.queue) > 4:
            self.queue.pop(0)
        if len(self.queue) != 4:
            return
        if self.start is None:
            stack = np.stack([spatial(f, self.window, self.chroma) for f in self.queue], axis=-1)
            s = q(upper_median4(stack))
            self.start = np.stack([s, s, s, np.full_like(s, 255)], axis=-1)
        if self.slots is None:
            self.slots = [f.copy() for f in self.queue]
            self.ring = 0
            self.uniform = 0
        else:
            self.slots[self.ring] = frame.copy()
            self.uniform = self.ring
            self.ring = (self.ring + 1) % 4

    def dispatch(self):
        if self.slots is None:
            return None
        u = self.uniform
        fi = spatial(self.slots[u], self.window, self.chroma)
        qi = q(fi)
        self.slots[u] = np.stack([qi, qi, qi, np.full_like(qi, 255)], axis=-1)
        stack = np.stack([intensity(s[..., :3], self.chroma, gray=False) for s in self.slots], axis=-1)
        med = upper_median4(stack)
        orig = U_LUT[self.start[..., 0]]
        diff = (orig - med).astype(F32)
        return epilogue(diff, self.filter, self.k, self.colorize)


# --------------------------------------------------------------------------
# dips_alt DiPsCompute (dips_alt/src/dips_compute/mod.rs:243-647,
# dips_alt/src/dips_compute/shaders/pre_compute_shader.wgsl)
# --------------------------------------------------------------------------

def alt_spatial(img: np.ndarray, window: int, chroma: int) -> np.ndarray:
    """dips_alt spatial_median_filter (:134-186): the (2h)^2 window values and
    W^2 - (2h)^2 zeros sorted, element W^2/2 + 1 (no +1 entry, unlike dips)."""
    I = intensity(img[..., :3], chroma, gray=False)
    if window == 1:
        return I
    h, w = I.shape
    hw = window // 2
    size = window * window
    shifted = []
    for i in range(-hw, hw):        # x offset
        for j in range(-hw, hw):    # y offset
            ys, xs = np.arange(h) + j, np.arange(w) + i
            ok = ((ys >= 0) & (ys < h))[:, None] & ((xs >= 0) & (xs < w))[None, :]
            sub = I[np.clip(ys, 0, h - 1)][:, np.clip(xs, 0, w - 1)]
            shifted.append(np.where(ok, sub, F32(0.0)).astype(F32))
    vals = np.stack(shifted, axis=-1)
    pad = np.zeros((h, w, size - vals.shape[-1]), dtype=F32)
    return np.sort(np.concatenate([vals, pad], axis=-1), axis=-1)[..., size // 2 + 1].astype(F32)


def alt_temporal(stack: np.ndarray) -> np.ndarray:
    """pre_compute_main's sort (:212-227) of the n filtered values inside a
    zero-filled 16-entry array, element n/2: for n < 16 the sort spans one
    trailing zero, for n = 16 (index 16 clamped) it is the plain sort."""
    n = stack.shape[-1]
    if n < 16:
        stack = np.concatenate([stack, np.zeros(stack.shape[:-1] + (1,), dtype=F32)], axis=-1)
    return np.sort(stack, axis=-1)[..., n // 2].astype(F32)


class AltCompute:
    """numpy twin of DiPsCompute::send_frame (mod.rs:498-646)."""

    def __init__(self, num_textures, width, height, colorize=True, window=1, scalar=5.0,
                 filter_type=0, chroma=0):
        self.n = int(num_textures)
        self.w, self.h = int(width), int(height)
        self.colorize = bool(colorize)
        self.window = int(window)
        self.k = float(np.float32(scalar))
        self.filter = int(filter_type)
        self.chroma = int(chroma)
        self.slots = [np.zeros((self.h, self.w, 4), np.uint8) for _ in range(self.n)]
        self.snap = np.zeros((self.h, self.w), np.uint8)
        self.idx = 0

    def send_frame(self, frame, snapshot=False):
        self.slots[self.idx] = np.asarray(frame, np.uint8).reshape(self.h, self.w, 4).copy()
        self.idx = (self.idx + 1) % self.n
        med = alt_temporal(np.stack([alt_spatial(s, self.window, self.chroma) for s in self.slots],
                                    axis=-1))
        if snapshot:
            s = q(med)
            self.snap = s
            return np.stack([s, s, s, np.full_like(s, 255)], axis=-1)
        diff = (U_LUT[self.snap] - med).astype(F32)
        return epilogue(diff, self.filter, self.k, self.colorize)

    def run(self, frames, markers=()):
        """run_dips_on_file's loop (dips_alt/src/lib.rs:588-683)."""
        index, overall, outs = 0, 0, []
        for f in frames:
            outs.append(self.send_frame(f, snapshot=(index == 2)))
            if index <= 2:
                index += 1
            overall += 1
            if overall in markers:
                index = 0
        return np.stack(outs) if outs else np.zeros((0, self.h, self.w, 4), np.uint8)
