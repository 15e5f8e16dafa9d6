"""Frame-range sharding of the difference series over one process per GPU.

The series path partitions by frames: once the reference is known, frames
are independent.  Rank k owns the contiguous global frames
[k*N/G, (k+1)*N/G).  The only exchanges are
  * 'overall': the reference frame, broadcast once from rank 0;
  * 'per-frame': the halo frame (global index start-1), sent by rank k-1 to
    rank k (one point-to-point transfer per batch);
  * the per-frame series (32 B per frame), reassembled on rank 0 by ONE
    gather (RCCL over xGMI with the "nccl" backend; gloo in the CPU tests).
No collective touches the frame data itself.

The per-rank compute is a callable so that the CPU tests can drive the same
protocol with the oracle over gloo; the product passes the HIP operator
(DiffSeriesOperator.run_device) and never a CPU function.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist

SERIES_COLS = 4  # sad, sj, count, si_fixed


def frame_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous frame range of `rank` (balanced to within one frame)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return (n_total * rank) // world, (n_total * (rank + 1)) // world


def frame_ranges(n_total: int, world: int) -> List[Tuple[int, int]]:
    return [frame_range(n_total, world, r) for r in range(world)]


def broadcast_reference(ref: torch.Tensor, src: int = 0, group=None) -> torch.Tensor:
    """'overall' mode: the reference frame from rank `src` to every rank."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.broadcast(ref, src=src, group=group)
    return ref


def exchange_halo(local_frames: torch.Tensor, halo: torch.Tensor, group=None) -> Optional[torch.Tensor]:
    """'per-frame' mode: send this rank's last frame to rank+1 and receive
    rank-1's last frame into `halo`.  Returns the halo (None on rank 0)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return None
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    ops = []
    if rank + 1 < world and local_frames.shape[0] > 0:
        ops.append(dist.P2POp(dist.isend, local_frames[-1].contiguous(), rank + 1, group))
    if rank > 0:
        ops.append(dist.P2POp(dist.irecv, halo, rank - 1, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return halo if rank > 0 else None


def start_halo(local_frames: torch.Tensor, halo: torch.Tensor, group=None) -> List:
    """Asynchronous form of exchange_halo: posts the send of this rank's last
    frame and the receive of rank-1's last frame, returns the work handles
    (empty on a single rank).  Frames 1.. of the shard do not depend on the
    halo, so their compute can run while the transfer is in flight."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return []
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    ops = []
    if rank + 1 < world and local_frames.shape[0] > 0:
        ops.append(dist.P2POp(dist.isend, local_frames[-1].contiguous(), rank + 1, group))
    if rank > 0:
        ops.append(dist.P2POp(dist.irecv, halo, rank - 1, group))
    return dist.batch_isend_irecv(ops) if ops else []


def per_frame_overlapped(local_frames: torch.Tensor, halo: torch.Tensor, series: torch.Tensor,
                         compute: Callable[[torch.Tensor, Optional[torch.Tensor], torch.Tensor], None],
                         group=None) -> None:
    """'per-frame' batch with the halo transfer hidden behind the compute of
    frames 1..n-1 (each against its local predecessor); frame 0 is computed
    against the received halo (or itself on rank 0) once the transfer lands."""
    works = start_halo(local_frames, halo, group)
    n = local_frames.shape[0]
    if n > 1:
        compute(local_frames[1:], local_frames[0], series[1:])
    for w in works:
        w.wait()
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    compute(local_frames[:1], halo if rank > 0 else None, series[:1])


class SeriesGather:
    """Reassemble the per-rank series on rank 0 with one gather.

    Shards may differ by one frame; every rank pads to the largest shard so
    the gather moves equal-size buffers, and rank 0 trims the padding."""

    def __init__(self, n_total: int, device: torch.device, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.ranges = frame_ranges(n_total, self.world)
        self.max_n = max(e - s for s, e in self.ranges)
        self.n_total = n_total
        self.send = torch.zeros((self.max_n, SERIES_COLS), dtype=torch.int64, device=device)
        self.recv = ([torch.zeros_like(self.send) for _ in range(self.world)]
                     if self.rank == 0 else None)

    def __call__(self, local_series: torch.Tensor) -> Optional[torch.Tensor]:
        n = local_series.shape[0]
        if self.world == 1:
            return local_series
        if n == self.max_n:
            send = local_series
        else:
            self.send[:n].copy_(local_series)
            send = self.send
        dist.gather(send, self.recv, dst=0, group=self.group)
        if self.rank != 0:
            return None
        return torch.cat([buf[: e - s] for buf, (s, e) in zip(self.recv, self.ranges)], dim=0)


def _comm_device(device: torch.device, group=None) -> torch.device:
    """Where collective tensors live: the GPU under RCCL ("nccl"), the host
    under gloo."""
    if dist.is_initialized() and dist.get_backend(group) == "nccl":
        return device
    return torch.device("cpu")


def check_frames(n_total: int, world: int, n_random: int = 8, seed: int = 0x5EED) -> List[int]:
    """Global frames rank 0 re-derives after a sharded step: the first and
    last frame, both sides of every shard boundary (k*F-1, k*F, k*F+1) and
    `n_random` frames drawn with a fixed seed."""
    import numpy as np
    picks = {0, n_total - 1}
    for s, _ in frame_ranges(n_total, world)[1:]:
        picks.update((s - 1, s, s + 1))
    if n_total > 0:
        picks.update(int(g) for g in np.random.default_rng(seed).integers(0, n_total, n_random))
    return sorted(g for g in picks if 0 <= g < n_total)


def verify_sharded_series(op, *, width: int, height: int, seed: int, n_total: int, per_frame: bool,
                          local_series: torch.Tensor, ref: Optional[torch.Tensor],
                          gathered: Optional[torch.Tensor], device: torch.device,
                          n_random: int = 8, group=None) -> dict:
    """Self-check of one sharded step over frames the shared generator makes
    (op.synth_device), run after the timed steps at any world size.

    * every rank regenerates its first two frames (and, per-frame, the frame
      before them) and requires its own first two series entries to match a
      fresh launch: entry 0 against the received halo ('per-frame', rank > 0)
      or the broadcast reference ('overall'), whose bytes must also equal the
      regenerated frame -- this is what tests the RCCL halo / broadcast;
    * rank 0 regenerates every global frame of check_frames() with its
      reference and requires the gathered series rows to match -- this tests
      the gather's ordering and padding.

    `op` is a DiffSeriesOperator of the batch's format, mode and tau; `ref`
    is the halo ('per-frame') or the reference ('overall') the step used.
    Returns the same {"frames_checked", "equal", "local_equal",
    "gathered_equal"} on every rank."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    s, e = frame_range(n_total, world, rank)
    n = e - s
    c = int(op.fmt)
    shape = (height, width) if c == 1 else (height, width, c)

    def synth(t0: int, count: int) -> torch.Tensor:
        buf = torch.empty((count,) + shape, dtype=torch.uint8, device=device)
        op.synth_device(buf, width, height, seed, t0)
        return buf

    def series_of(frames: torch.Tensor, r: Optional[torch.Tensor]) -> torch.Tensor:
        out = torch.zeros((frames.shape[0], SERIES_COLS), dtype=torch.int64, device=device)
        op.run_device(frames, out, ref=r)
        return out

    # -- local: this rank's first entries and the reference it received ------
    local_ok = True
    k = min(n, 2)
    if k > 0:
        mine = local_series[:k].to(device)
        if per_frame:
            if s > 0:
                buf = synth(s - 1, k + 1)
                want = series_of(buf, None)[1:]
                local_ok = ref is not None and torch.equal(ref.to(device).reshape(shape), buf[0])
            else:
                want = series_of(synth(0, k), None)
        else:
            frame0 = synth(0, 1)[0]
            local_ok = ref is not None and torch.equal(ref.to(device).reshape(shape), frame0)
            want = series_of(synth(s, k), frame0)
        local_ok = bool(local_ok) and bool(torch.equal(mine, want))
    cdev = _comm_device(device, group)
    # [ranks that failed, frames checked], summed over ranks
    flag = torch.tensor([0 if local_ok else 1, k], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(flag, group=group)
    all_local_ok = int(flag[0]) == 0

    # -- global: rank 0 re-derives boundary and random rows of the gather -----
    picks = check_frames(n_total, world, n_random)
    res = torch.tensor([0, len(picks)], dtype=torch.int64, device=cdev)
    if rank == 0:
        got = gathered.to(device)[picks] if gathered is not None and gathered.shape[0] == n_total else None
        if per_frame:
            # pairs (g-1, g) in one per-frame launch: the entry at 2i+1 is g's
            buf = torch.empty((2 * len(picks),) + shape, dtype=torch.uint8, device=device)
            for i, g in enumerate(picks):
                if g == 0:  # frame 0 against itself
                    op.synth_device(buf[2 * i:2 * i + 1], width, height, seed, 0)
                    op.synth_device(buf[2 * i + 1:2 * i + 2], width, height, seed, 0)
                else:
                    op.synth_device(buf[2 * i:2 * i + 2], width, height, seed, g - 1)
            want = series_of(buf, None)[1::2]
        else:
            buf = torch.empty((len(picks),) + shape, dtype=torch.uint8, device=device)
            for i, g in enumerate(picks):
                op.synth_device(buf[i:i + 1], width, height, seed, g)
            want = series_of(buf, synth(0, 1)[0])
        res[0] = 1 if got is not None and torch.equal(got, want) else 0
        del buf
    if world > 1:
        dist.broadcast(res, src=0, group=group)
    gathered_ok = bool(int(res[0]) == 1)
    return {"frames_checked": int(res[1]) + int(flag[1]), "equal": all_local_ok and gathered_ok,
            "local_equal": all_local_ok, "gathered_equal": gathered_ok, "global_frames": picks}


# ---------------------------------------------------------------------------
# dips-compat ComputeState over frame ranges ("dips-compat T=4
# needs a 3-frame halo").  Output frame t depends on the start texture S
# (built from frames 0..3) and, through the temporal ring, on frames
# t-3..t; so rank k > 0 needs S (broadcast once from rank 0) and the raw
# frames s_k-3..s_k-1 (the last three of rank k-1), and resumes there
# (ComputeState.resume / dips_compat_resume).
# ---------------------------------------------------------------------------
COMPAT_HALO = 3


def start_compat_halo(local_frames: torch.Tensor, halo: torch.Tensor, group=None) -> List:
    """Post the send of this rank's last 3 frames to rank+1 and the receive
    of rank-1's last 3 frames into `halo` ([3, H, W, 4]); returns the works."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return []
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    ops = []
    if rank + 1 < world:
        if local_frames.shape[0] < COMPAT_HALO:
            raise ValueError("every shard of the dips-compat path needs >= 3 frames")
        ops.append(dist.P2POp(dist.isend, local_frames[-COMPAT_HALO:].contiguous(), rank + 1, group))
    if rank > 0:
        ops.append(dist.P2POp(dist.irecv, halo, rank - 1, group))
    return dist.batch_isend_irecv(ops) if ops else []


def _check_compat_shards(local_frames: torch.Tensor, t0: int, rank: int, world: int, group=None) -> None:
    """Validate every rank's (t0, n) on every rank before any frame moves, so
    that a bad layout raises the same error everywhere instead of leaving the
    other ranks blocked in a send, receive or broadcast."""
    mine = torch.tensor([t0, local_frames.shape[0]], dtype=torch.int64, device=local_frames.device)
    if world > 1:
        parts = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine, group=group)
        shards = [(int(p[0]), int(p[1])) for p in parts]
    else:
        shards = [(int(mine[0]), int(mine[1]))]
    if shards[0][0] != 0:
        raise ValueError("rank 0 owns the first frames")
    for r, (s, n) in enumerate(shards):
        if r > 0 and s < 7:
            raise ValueError(f"ranks after the first must start at global frame >= 7 (rank {r} starts at {s})")
        if r + 1 < world and n < COMPAT_HALO:
            raise ValueError("every shard of the dips-compat path needs >= 3 frames")


def compat_sharded(local_frames: torch.Tensor, t0: int, *,
                   callback_batch: Callable[[torch.Tensor], torch.Tensor],
                   start_texture: Callable[[torch.Tensor], None],
                   resume: Callable[[torch.Tensor, torch.Tensor, int], None],
                   start_buf: torch.Tensor, halo_buf: torch.Tensor, group=None) -> torch.Tensor:
    """frame_callback over this rank's frames (global t0 .. t0+n-1) with the
    outputs a single ComputeState would give.  Rank 0 starts from frame 0,
    builds S at its 4th frame and broadcasts it; every other rank resumes
    from S and the halo (t0 >= 7 there).  callback_batch(frames) returns the
    outputs of consecutive frame_callback calls; start_texture(buf) fills S;
    resume(S, halo, t0) sets the state.  Returns this rank's outputs."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    _check_compat_shards(local_frames, t0, rank, world, group)
    works = start_compat_halo(local_frames, halo_buf, group)
    if rank == 0:
        head = callback_batch(local_frames[:4])  # frames 0..3: passthrough, then S
        start_texture(start_buf)
    if world > 1:
        dist.broadcast(start_buf, src=0, group=group)
    if rank == 0:
        tail = callback_batch(local_frames[4:]) if local_frames.shape[0] > 4 else head[:0]
        for w in works:
            w.wait()
        return torch.cat([head, tail])
    for w in works:
        w.wait()
    resume(start_buf, halo_buf, t0)
    return callback_batch(local_frames)


# ---------------------------------------------------------------------------
# dips_alt run loop over frame ranges.  Output frame t reads the N texture
# slots (frames t-N+1..t) and the snapshot texture, which the last snapshot
# frame s < t set from the slots it saw (frames s-N+1..s); the snapshot
# flags follow from the refresh markers alone (alt.run_loop_flags).  Rank k
# therefore needs the raw frames s-N+1..s and t0-N..t0-1 from the ranks that
# own them, replays them through a fresh DiPsCompute (snapshot on s,
# outputs discarded) and continues with its own frames and flags -- no new
# operator state beyond what send_frames already keeps.
# ---------------------------------------------------------------------------
def alt_replay_frames(t0: int, flags, num_textures: int) -> Tuple[List[int], List[bool]]:
    """Global frames (>= 0) rank starting at t0 replays, with their flags."""
    if t0 == 0:
        return [], []
    prior = [t for t in range(t0) if flags[t]]
    frames, fl = [], []
    if prior:
        s = prior[-1]
        for g in range(max(0, s - num_textures + 1), s + 1):
            frames.append(g)
            fl.append(g == s)
    for g in range(max(0, t0 - num_textures), t0):
        frames.append(g)
        fl.append(False)
    return frames, fl


def alt_sharded(local_frames: torch.Tensor, t0: int, n_total: int, flags, num_textures: int, *,
                send_frames: Callable[[torch.Tensor, List[bool]], torch.Tensor], group=None) -> torch.Tensor:
    """dips_alt run loop over this rank's frames (global t0..), identical to
    one DiPsCompute that saw every frame.  `flags`: run_loop_flags of all
    n_total frames; send_frames(frames, flags) drives this rank's fresh
    DiPsCompute and returns the outputs.  Needed frames travel point to
    point from their owners (one op per frame, posted in increasing frame
    order on both sides)."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    ranges = frame_ranges(n_total, world)
    owner = lambda g: next(r for r, (a, b) in enumerate(ranges) if a <= g < b)  # noqa: E731
    ops, recv = [], {}
    for j in range(1, world):
        need, _ = alt_replay_frames(ranges[j][0], flags, num_textures)
        for g in sorted(set(need)):
            o = owner(g)
            if o == j:
                continue
            if o == rank:
                ops.append(dist.P2POp(dist.isend, local_frames[g - t0].contiguous(), j, group))
            elif j == rank:
                buf = torch.empty_like(local_frames[0])
                recv[g] = buf
                ops.append(dist.P2POp(dist.irecv, buf, o, group))
    works = dist.batch_isend_irecv(ops) if ops else []
    for w in works:
        w.wait()
    need, fl = alt_replay_frames(t0, flags, num_textures)
    if need:
        frames = [recv[g] for g in need]
        halo_len = t0 - max(0, t0 - num_textures)
        if halo_len < num_textures and len(need) > halo_len:
            # t0 < N: the single loop still has N - t0 zero (never written)
            # slots at frame t0, evicted before frame 0's slot; the snapshot
            # replay filled them, so push that many all-zero frames (a zero
            # texel is what wgpu's zero-initialised slot reads as) before the
            # halo, in the single loop's eviction order
            zero = torch.zeros_like(local_frames[0])
            k = len(need) - halo_len
            pad = num_textures - halo_len
            frames = frames[:k] + [zero] * pad + frames[k:]
            fl = fl[:k] + [False] * pad + fl[k:]
        replay = torch.stack(frames)
        send_frames(replay, fl)  # state only: slots and snapshot as at global frame t0
    return send_frames(local_frames, [bool(f) for f in flags[t0:t0 + local_frames.shape[0]]])


def sharded_series(local_frames: torch.Tensor, *, per_frame: bool, n_total: int,
                   compute: Callable[[torch.Tensor, Optional[torch.Tensor], torch.Tensor], None],
                   reference: Optional[torch.Tensor] = None, group=None,
                   gather: Optional[SeriesGather] = None) -> Optional[torch.Tensor]:
    """One batch of the sharded path.

    local_frames: this rank's frames [n_k, ...]; reference: 'overall' mode's
    reference (already broadcast); compute(frames, ref, series_out) fills
    series_out [n_k, 4] (int64).  Returns the full series on rank 0."""
    device = local_frames.device
    series = torch.zeros((local_frames.shape[0], SERIES_COLS), dtype=torch.int64, device=device)
    if per_frame:
        halo = torch.empty_like(local_frames[0])
        ref = exchange_halo(local_frames, halo, group)
    else:
        ref = reference
    compute(local_frames, ref, series)
    gather = gather or SeriesGather(n_total, device, group)
    return gather(series)
