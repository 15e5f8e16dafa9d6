#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X DiPs difference-series path.

Metric (BASELINE.json): frames/s + achieved HBM GB/s (% of roofline), 4K RGB8,
1/2/4/8 GPUs.  Workload at N GPUs: BASELINE.json configs[2] per GPU --
3840x2160 RGB8 synthetic frames, 5000 per GPU, 'per-frame' mode -- weakly
scaled: rank k owns global frames [k*F, (k+1)*F), receives the halo frame
k*F-1 from rank k-1 (RCCL send/recv) and rank 0 gathers the per-frame series
(one RCCL gather).  `--mode overall` runs configs[3]'s mode instead (the
reference frame is broadcast once at setup).

A step = one pass of the hot path over the rank's resident frame batch:
series kernel + reduction (+ halo exchange + series gather when N > 1).
At N > 1 the step is ONE call of the library's native sharded entry point,
dips_diff_series_sharded (shard_abi.hip), over an RCCL communicator the
ranks build from a unique id passed over the torch process group: the halo
ncclSend/ncclRecv beside the series launch and one ncclGather of the series,
all inside libdips_hip.so.  (DIPS_BENCH_SHARD=torch runs the older
Python-level protocol of dips_amd.shard over torch.distributed instead.)
Frames are generated into HBM by the shared integer generator before timing.

After the timed steps, at every N (the driver's 8-GPU run included):
  * "check": every rank re-derives its first series entries against the halo
    / reference it received, rank 0 the gathered rows at every shard boundary
    and 8 random frames (dips_amd.shard.verify_sharded_series); a mismatch
    makes the process exit non-zero after printing the line;
  * "configs3" / "configs4": BASELINE.json configs[3] ('overall', reference
    broadcast, 5000 4K frames per GPU) and configs[4] (7680x4320, tau 8/255,
    1250 frames per GPU) on the same ranks, regenerated into the same
    resident buffer, each with frames/s, roofline fraction, RCCL times and
    its own check;
  * at N = 1 also "per_frame_call": the reference's own pattern, one 4K RGBA8
    frame per dips_frame_callback from pageable host memory.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE).
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import traceback
from datetime import timedelta

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/s + achieved HBM GB/s (% of roofline), 4K RGB8, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md "Chip-level parameters")
SEED = 0xD1B5


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames-per-gpu", type=int, default=5000)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--mode", choices=["per-frame", "overall"], default="per-frame")
    ap.add_argument("--tau", type=float, default=8.0 / 255.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the pcie_inclusive sample (profiling runs: its chunk launches of the series "
                         "kernel would mix into the kernel statistics)")
    ap.add_argument("--check", action="store_true",
                    help="rank 0 recomputes the series of all N*F frames in one single-device launch "
                         "and requires the gathered series to equal it (functional check of the N>1 path)")
    ap.add_argument("--no-map", action="store_true", help="skip the map_variant measurement")
    ap.add_argument("--no-tau0", action="store_true", help="skip the tau = 0 leg at the headline shape")
    ap.add_argument("--map-frames", type=int, default=2500,
                    help="frames of the map_variant launch (frames + maps stay resident beside the batch)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU work of the cpu_baseline sample")
    ap.add_argument("--no-check", action="store_true",
                    help="skip the self-check after the timed steps (profiling runs only: its small launches of "
                         "the series kernel would mix into the kernel statistics)")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the configs[3] / configs[4] legs (profiling runs)")
    ap.add_argument("--leg-steps", type=int, default=5, help="timed steps of each configs[3] / configs[4] leg")
    ap.add_argument("--no-per-frame-call", action="store_true", help="skip the per_frame_call leg")
    ap.add_argument("--no-placement-probe", action="store_true",
                    help="one plain allocation of the frame batch instead of the probed choice between two "
                         "candidate placements (tools/placement.py resident_frames)")
    ap.add_argument("--per-frame-calls", type=int, default=200,
                    help="timed dips_frame_callback calls of the per_frame_call leg (4K RGBA8)")
    ap.add_argument("--dump-series", default=None,
                    help="rank 0 saves the gathered series of the timed step (uint64 [N*F, 4]) to this .npy, and "
                         "each configs leg's beside it as <stem>_<leg>.npy (tests compare them with the oracle)")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds a collective may wait before the process group fails (init_process_group timeout)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="HBM traffic per launch measured by profiles/collect_pmc.sh")
    return ap.parse_args()


def _series_isi(tau: float) -> int:
    """The intensity-sum form run_series_device (series_abi.hip) picks: 0 (the
    exact f64 sum) below tau = 2^-5, else 1 (the integer sum)."""
    return 1 if tau >= 0.03125 else 0


def _v2_kernel_name(per_frame: bool, tau: float, with_map: bool = False) -> str:
    """The series_v2_kernel instantiation the library runs for an aligned RGB8
    batch (series_v2.hip: <C, CH, U, PF, MAP, ALIGN, ISI>; U = 5 for RGB8), spelled as
    rocprofv3 prints it (ISI is an int template argument)."""
    b = lambda v: "true" if v else "false"  # noqa: E731
    return f"series_v2_kernel<3, 0, 5, {b(per_frame)}, {b(with_map)}, false, {_series_isi(tau)}>"


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _time_oracle(lib, frames, mode, tau, threads, target_s, max_passes=400):
    """Run the oracle series over `frames` on `threads` host threads until
    about target_s seconds have been timed; returns (frames/s, passes, s, out4)."""
    from oracle import oracle
    passes, out4 = 0, None
    t = time.perf_counter()
    while True:
        out4, _, _ = oracle.series(frames, mode=mode, tau=tau, nthreads=threads, lib=lib)
        passes += 1
        dt = time.perf_counter() - t
        if dt >= target_s or passes >= max_passes:
            break
    return frames.shape[0] * passes / dt, passes, dt, out4


def cpu_baseline(frames_dev, series_dev, mode: int, tau: float, target_s: float, op_gray=None, pf_sample=None):
    """The oracle ('port' of the reference semantics; the reference itself has
    no CPU loop) timed on this host's cores on a bounded
    prefix of the same frames (per-frame cost is constant): all usable cores
    (the headline baseline), the box's CPU share, and one core
    ("1 thread and all cores"); plus configs[0] (640x480 gray8,
    300 frames, 'overall') at one core and all cores."""
    from oracle import oracle
    try:
        path = oracle.build(native=True)
        lib = oracle.load(path)
        build = "gcc -O3 -march=native -ffp-contract=off"
    except Exception:  # pragma: no cover - no compiler on the box
        lib = oracle.load()
        build = "gcc -O3 -ffp-contract=off (prebuilt)"
    host = _host_cpu()
    all_threads = max(1, host["usable_cpus"] or os.cpu_count() or 1)
    share = max(1, min(all_threads, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    # bounded host sample: enough frames for one per thread (<= 384 4K
    # frames, 9.6 GB), passed over repeatedly until ~target_s is timed
    n = min(frames_dev.shape[0], max(64, min(all_threads, 384)))
    sample = frames_dev[:n].cpu().numpy()
    v_all, p_all, dt_all, out4 = _time_oracle(lib, sample, mode, tau, all_threads, target_s)
    # the same sample doubles as a parity check of the timed GPU series
    gpu = series_dev[:n].cpu().numpy().view(np.uint64)
    matches = bool(np.array_equal(gpu, out4))
    v_share, p_share, dt_share, o2 = _time_oracle(lib, sample[: min(n, 4 * share)], mode, tau, share,
                                                  max(2.0, target_s / 4))
    matches = matches and bool(np.array_equal(o2, out4[: o2.shape[0]]))
    # one core: 4 frames a pass (mode 'per-frame' needs the frame before
    # each, so the pass is the prefix), at least 2.5 s
    v1, p1, dt1, o1 = _time_oracle(lib, sample[:4], mode, tau, 1, 2.5)
    matches = matches and bool(np.array_equal(o1, out4[:4]))
    # the reported baseline is the fastest thread count measured (on the
    # GPU boxes the cgroup CPU quota makes all 256 visible CPUs slower than
    # the box's share); every figure is kept beside it
    all_cores = {"value": round(v_all, 3), "unit": "frames/s", "cores": all_threads,
                 "sample": f"first {n} frames x {p_all} passes, {dt_all:.2f} s"}
    box_share = {"value": round(v_share, 3), "unit": "frames/s", "cores": share,
                 "sample": f"first {min(n, 4 * share)} frames x {p_share} passes, {dt_share:.2f} s"}
    best = all_cores if v_all >= v_share else box_share
    res = {"value": best["value"], "unit": "frames/s", "cores": best["cores"], "kind": "port",
           "sample": f"synthetic 4K RGB8 frames of the same batch, series only (oracle/dips_oracle.c, {build}, "
                     f"threads over frame ranges): {best['sample']}; the fastest of all usable cores "
                     f"({all_threads} threads) and the box's share ({share} threads)",
           "all_cores": all_cores,
           "box_share": box_share,
           "single_core": {"value": round(v1, 3), "unit": "frames/s", "cores": 1,
                           "sample": f"first 4 frames x {p1} passes, {dt1:.2f} s"},
           "host": host,
           "series_matches_gpu": matches}
    # configs[0]: the reference's own CPU-runnable case (BASELINE.json configs[0])
    try:
        c0 = oracle.synth(1, 640, 480, SEED, 0, 300, lib=lib)
        r1, q1, d1, w1 = _time_oracle(lib, c0, 0, 0.0, 1, 2.5)
        ra, qa, da, wa = _time_oracle(lib, c0, 0, 0.0, min(all_threads, 300), 2.5)
        cfg0 = {"workload": "640x480 gray8 synthetic 300-frame clip, 'overall', tau=0 (BASELINE.json configs[0])",
                "single_core": {"value": round(r1, 1), "unit": "frames/s", "cores": 1,
                                "sample": f"300 frames x {q1} passes, {d1:.2f} s"},
                "all_cores": {"value": round(ra, 1), "unit": "frames/s", "cores": min(all_threads, 300),
                              "sample": f"300 frames x {qa} passes, {da:.2f} s"},
                "threads_agree": bool(np.array_equal(w1, wa))}
        if op_gray is not None:
            cfg0["gpu"] = op_gray(c0, wa)
        res["config0"] = cfg0
    except Exception as e:  # report, never hide
        res["config0"] = {"failed": str(e)}
    # the per-frame call pattern: the oracle's ComputeState frame_callback
    # (one core) over the first frames of the per_frame_call leg; its outputs
    # must equal the GPU's
    if pf_sample is not None:
        try:
            frames_pf, want_pf = pf_sample
            n_pf, h_pf, w_pf = frames_pf.shape[:3]
            cs = oracle.ComputeState(False, 1, 5.0, 255, 0)
            same = True
            t = time.perf_counter()
            for k in range(n_pf):
                o = oracle.frame_callback(w_pf, h_pf, frames_pf[k], cs)
                same = same and bool(np.array_equal(o, want_pf[k]))
            dt = time.perf_counter() - t
            res["per_frame_call"] = {"value": round(n_pf / dt, 3), "unit": "frames/s", "cores": 1,
                                     "sample": f"frame_callback of the first {n_pf} 4K RGBA8 frames of the "
                                               f"per_frame_call leg, {dt:.2f} s (oracle ComputeState)",
                                     "outputs_equal_gpu": same}
        except Exception as e:  # report, never hide
            res["per_frame_call"] = {"failed": str(e)}
    return res


def _host_cpu() -> dict:
    """CPU model and logical CPU count of the host the baseline ran on."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": os.cpu_count(), "usable_cpus": usable, "cgroup_cpu_quota": quota}


def _cgroup_cpu_stat() -> dict:
    """The cgroup's CPU accounting (cgroup v2 cpu.stat: usage_usec,
    nr_throttled, throttled_usec), {} where unreadable: a delta over a leg
    gives the CPUs it kept busy and the time the CPU quota throttled it."""
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if len(line.split()) == 2)}
    except (OSError, ValueError):
        return {}


def _lib_sha256() -> str:
    """sha256 of the loaded HIP library: profiles/pmc_traffic.json is used
    for roofline.traffic only when it was collected with this very build."""
    import hashlib
    from dips_amd import _lib as L
    path = L.LIB_PATH
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _config0_gpu(torch, frames_host, want):
    """configs[0] on the GPU beside its CPU figures: the 300-frame 640x480
    gray8 clip resident in HBM, 'overall', tau 0; series checked against the
    oracle's."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    op = DiffSeriesOperator(PixelFormat.Gray8, Mode.Overall, 0.0, time_kernel=True)
    try:
        dev = torch.from_numpy(frames_host).cuda()
        ser = torch.zeros((dev.shape[0], 4), dtype=torch.int64, device="cuda")
        op.run_device(dev, ser)
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        reps = 20
        t = time.perf_counter()
        for _ in range(reps):
            op.run_device(dev, ser)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / reps
        kms, n = op.kernel_time()
        kms /= max(n, 1)
        ok = bool(np.array_equal(ser.cpu().numpy().view(np.uint64), want))
    finally:
        op.close()
    nb = frames_host.size
    return {"frames_per_s": round(frames_host.shape[0] / wall, 1), "kernel_ms": round(kms, 4),
            "kernel_GBps": round(nb / (kms / 1e3) / 1e9, 1), "series_matches_oracle": ok,
            "note": "92 MB batch: launch-bound (a 300-frame 640x480 clip is ~0.03 ms of HBM streaming)"}


def _power_sampler(torch, local):
    """amdsmi reader of this rank's GPU (tools/power_probe.py, read-only
    queries), not started: legs take one reading right before and one right
    after themselves (_power_leg), so nothing runs beside them; None where
    amdsmi is unavailable."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from power_probe import Sampler
        bus = torch.cuda.get_device_properties(local).pci_bus_id
        smp = Sampler(pci_bus=bus)
        return smp if len(smp.handles) == 1 else None
    except Exception:  # report nothing rather than fail the bench
        return None


def _power_leg(smp, run, frames, what):
    """run() between two readings of the socket energy counter, the PPT
    residency accumulator and the gfx clocks: average W, PPT throttle
    residency, clock before / after and mJ per frame (`frames` = the frames
    run() read) of exactly that interval; (run()'s result, report or None)."""
    if smp is None:
        return run(), None
    try:
        smp.sample()
        ta = smp.rows[-1][0]
    except Exception:
        return run(), None
    res = run()
    try:
        smp.sample()
        tb = smp.rows[-1][0]
        g = smp.window(ta, tb)[0]
        if not g or not g.get("avg_power_W_energy"):
            return res, None
        return res, {"avg_W": g["avg_power_W_energy"],
                     "gfxclk_MHz_before_after": [r[4] for r in smp.rows if ta <= r[0] <= tb],
                     "ppt_throttle_residency": g.get("ppt_residency_frac"),
                     "seconds": round(tb - ta, 3),
                     "mJ_per_frame": round(g["avg_power_W_energy"] * (tb - ta) / frames * 1e3, 4),
                     "source": f"amdsmi energy counter and PPT residency accumulator read right before and right "
                               f"after {what}, gfx clock at both readings (tools/power_probe.py)"}
    except Exception:
        return res, None


def _map_variant(torch, op_cls, frames, n, W, H, mode_pf, tau):
    """The north star's bit-exact output D_t = |F_t - R| materialised: the
    MAP=true series kernel over n resident frames (read F, write D), timed by
    the library's hipEvents; the series must equal the no-map run and the
    maps of two frames are checked against a torch recomputation."""
    from dips_amd import Mode, PixelFormat
    op = op_cls(PixelFormat.RGB8, Mode.PerFrame if mode_pf else Mode.Overall, tau, time_kernel=True)
    fb = W * H * 3
    try:
        fr = frames[:n]
        dmap = torch.empty_like(fr)
        ser_m = torch.zeros((n, 4), dtype=torch.int64, device=fr.device)
        ser_n = torch.zeros((n, 4), dtype=torch.int64, device=fr.device)
        op.run_device(fr, ser_m, map_out=dmap)  # warm
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        steps = 3
        t = time.perf_counter()
        for _ in range(steps):
            op.run_device(fr, ser_m, map_out=dmap)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / steps
        each = op.kernel_times()
        op.run_device(fr, ser_n)
        torch.cuda.synchronize()
        same = bool(torch.equal(ser_m, ser_n))
        ok = True
        for k in (1, n - 1):
            r = fr[k - 1] if mode_pf else fr[0]
            want = (fr[k].to(torch.int16) - r.to(torch.int16)).abs().to(torch.uint8)
            ok = ok and bool(torch.equal(dmap[k], want))
        kms = float(np.median(each))
        algo = 2 * n * fb
        return {"kernel": _v2_kernel_name(mode_pf, tau, with_map=True),
                "frames": n, "frames_per_s": round(n / (kms / 1e3), 1), "wall_frames_per_s": round(n / wall, 1),
                "kernel_ms_median": round(kms, 4), "launches": len(each),
                "algorithmic_bytes_per_launch": algo, "achieved_GBps": round(algo / (kms / 1e3) / 1e9, 1),
                "frac_of_8TBps": round(algo / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                "bytes_note": "2*W*H*C per frame: F_t read once + D_t written once (R is the previous frame, "
                              "already in registers)",
                "series_equals_nomap_run": same, "map_matches_torch": ok}
    finally:
        op.close()


def _tau0_leg(torch, smp, op_cls, frames, series_hl, mode_pf, tau_hl, steps, device=0):
    """The headline shape at tau = 0 (BASELINE.json configs[2] does not state
    tau): every pixel with dI > 0 counted, the exact f64 intensity sum
    (series_v2.hip ISI = 0) instead of the integer sum the headline's tau >=
    2^-5 admits; `steps` back-to-back launches between power readings.  Checks
    that need no oracle: SAD and SJ do not depend on tau (equal the headline
    series), count and SI at tau 0 are >= the headline's for every frame."""
    from dips_amd import Mode, PixelFormat
    F = frames.shape[0]
    fb = frames[0].numel()
    # N = 1 only (bench.py runs it there): one launch over the whole batch,
    # the headline's own path at one rank
    op = op_cls(PixelFormat.RGB8, Mode.PerFrame if mode_pf else Mode.Overall, 0.0, time_kernel=True, device=device)
    try:
        ser = torch.zeros((F, 4), dtype=torch.int64, device=frames.device)
        op.run_device(frames, ser)  # warm
        torch.cuda.synchronize()
        op.kernel_time(reset=True)

        def run():
            t = time.perf_counter()
            for _ in range(steps):
                op.run_device(frames, ser)
            torch.cuda.synchronize()
            return time.perf_counter() - t

        wall, pw = _power_leg(smp, run, F * steps, f"{steps} back-to-back tau = 0 launches")
        each = op.kernel_times()
        a = ser.cpu().numpy().view(np.uint64)
        b = series_hl.cpu().numpy().view(np.uint64)
        kms = float(np.median(each))
        ach = F * fb / (kms / 1e3) / 1e9
        return {"workload": f"the headline batch at tau = 0 ({'per-frame' if mode_pf else 'overall'})",
                "kernel": _v2_kernel_name(mode_pf, 0.0), "steps": steps,
                "frames_per_s": round(F * steps / wall, 1), "kernel_ms_median": round(kms, 4),
                "achieved_GBps": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "power": pw,
                "sad_sj_equal_headline": bool(np.array_equal(a[:, :2], b[:, :2])),
                "count_si_ge_headline": bool(np.all(a[:, 2:] >= b[:, 2:])),
                "note": f"headline tau = {tau_hl:.6g} runs the integer sum (ISI = 1); tau = 0 the f64 sum (ISI = 0)"}
    finally:
        op.close()


def _plain_allocation(placement, algo_bytes, kernel_ms):
    """roofline.plain_kernel_ms / plain_frac: the series kernel on the plain
    (first) allocation of the batch, next to the headline's kept one."""
    if placement.get("probe"):
        ms = float(placement["candidate_kernel_ms"][0])
        note = ("candidate 0 (the plain allocation): median of its probe launches; the headline ran on "
                f"candidate {placement['kept']}")
    else:
        ms = kernel_ms
        note = "no placement probe: the headline ran on the plain allocation"
    return {"plain_kernel_ms": round(ms, 4),
            "plain_frac": round(algo_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "plain_note": note}


def _devices(torch, dist, world, local):
    """PCI bus id of every rank's GPU (all_gather), so the line proves which
    devices ran."""
    props = torch.cuda.get_device_properties(local)
    mine = f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
    if world == 1:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


class _DamagingTransport:
    """The rehearsal's host transport with the halo rank 1 receives damaged
    on purpose (DIPS_BENCH_CORRUPT_HALO=1: the self-check must catch it)."""

    def __init__(self, inner, rank):
        self.inner, self.rank = inner, rank

    def broadcast(self, buf, root):
        self.inner.broadcast(buf, root)

    def sendrecv(self, send, to, recv, src):
        self.inner.sendrecv(send, to, recv, src)
        if recv is not None and self.rank == 1:
            recv[12345 % recv.size] ^= 0x5A

    def gather(self, send, recv, root):
        self.inner.gather(send, recv, root)


def _make_comm(torch, dist, backend, world, rank, local, corrupt_halo):
    """(communicator, note) of the native sharded path: RCCL over the ranks of
    the process group (backend "nccl", the unique id broadcast over it), or
    the host transport over gloo (the one-GPU rehearsal).  Every rank must get
    one; otherwise all release theirs and return (None, why)."""
    from dips_amd.comm import Comm, TorchHostTransport, rccl_from_process_group
    comm, err = None, None
    try:
        if backend == "nccl":
            comm = rccl_from_process_group(local)
        else:
            tr = TorchHostTransport()
            comm = Comm.host(_DamagingTransport(tr, rank) if corrupt_halo else tr, world, rank, local)
    except Exception as e:  # reported in the line, and the torch path runs instead
        err = f"{type(e).__name__}: {e}"
    flag = torch.tensor([0 if comm is not None else 1], dtype=torch.int64,
                        device=torch.device("cuda", local) if backend == "nccl" else "cpu")
    dist.all_reduce(flag)
    if int(flag[0]) != 0:
        if comm is not None:
            comm.close()
        log(f"rank {rank}: native communicator unavailable on {int(flag[0])} rank(s) ({err}); torch path")
        return None, {"failed": err or "on another rank"}
    kind = "rccl" if backend == "nccl" else f"host ({backend}, rehearsal)"
    log(f"rank {rank}: native sharded path over {comm!r}")
    return comm, {"transport": kind}


def _gather_objects(dist, world, obj):
    """Every rank's obj, in rank order (all_gather_object)."""
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def _max_over_ranks(torch, dist, world, dev, values):
    t = torch.tensor(values, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]


def _config_leg(torch, dist, buf, *, name, W, H, F, mode, tau, steps, world, rank, local, dev, check=True,
                dump=None, comm=None):
    """One more BASELINE.json config on the same ranks and the same resident
    buffer (regenerated in place, so HBM holds one batch at a time): 'overall'
    mode, the reference broadcast once (RCCL), each step the series kernel
    over the rank's F frames + one gather of the series -- one
    dips_diff_series_sharded call with `comm` (the native path); then the
    same self-check as the headline.  Returns its frames/s, roofline
    fraction, RCCL times and check."""
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat, shard

    fb = W * H * 3
    if F * fb > buf.numel():
        raise ValueError("leg does not fit the resident buffer")
    op = DiffSeriesOperator(PixelFormat.RGB8, mode, tau, time_kernel=True, device=local)
    try:
        frames = buf.view(-1)[: F * fb].view(F, H, W, 3)
        op.synth_device(frames, W, H, SEED, rank * F)
        series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
        ref = torch.empty((H, W, 3), dtype=torch.uint8, device=dev)
        native = comm is not None and world > 1
        if native:
            gathered = torch.zeros((world * F, 4), dtype=torch.int64, device=dev) if rank == 0 else None
        else:
            gather_t = shard.SeriesGather(world * F, dev)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = time.perf_counter()
        if mode == Mode.Overall:
            if native:
                op.shard_broadcast_device(comm, frames[0] if rank == 0 else None, ref)
            else:
                if rank == 0:
                    ref.copy_(frames[0])
                shard.broadcast_reference(ref)
        torch.cuda.synchronize()
        ref_ms = (time.perf_counter() - t) * 1e3

        def compute():
            if native:
                op.run_sharded(comm, frames, world * F, series, gathered,
                               ref=ref if mode == Mode.Overall else None, ref_resident=mode == Mode.Overall)
            elif mode == Mode.Overall:
                op.run_device(frames, series, ref=ref)
            elif world == 1:
                op.run_device(frames, series)
            else:
                shard.per_frame_overlapped(frames, ref, series, lambda fr, r, out: op.run_device(fr, out, ref=r))

        def gather(ser):
            return gathered if native else gather_t(ser)

        compute()
        gather(series)  # warm
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        final = None
        for _ in range(steps):
            compute()
            final = gather(series)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t
        kms, _ = op.kernel_time()
        # the gather alone, once more (its share of a step; inside the
        # sharded call on the native path, so not separable there)
        gather_ms = 0.0
        if not native:
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t = time.perf_counter()
            final = gather(series)
            torch.cuda.synchronize()
            gather_ms = (time.perf_counter() - t) * 1e3
        elapsed, kms, gather_ms, ref_ms = _max_over_ranks(torch, dist, world, dev,
                                                          [elapsed, kms / steps, gather_ms, ref_ms])
        chk = None
        if check:
            chk = shard.verify_sharded_series(op, width=W, height=H, seed=SEED, n_total=world * F,
                                              per_frame=(mode == Mode.PerFrame), local_series=series, ref=ref,
                                              gathered=final, device=dev)
            chk.pop("global_frames", None)
        if dump and rank == 0 and final is not None:
            np.save(dump, final.cpu().numpy().view(np.uint64))
        algo = F * fb
        ach = algo / (kms / 1e3) / 1e9
        return {"workload": name, "frames_per_gpu": F, "width": W, "height": H,
                "mode": "overall" if mode == Mode.Overall else "per-frame", "tau": round(tau, 6),
                "steps": steps, "frames_per_s": round(world * F * steps / elapsed, 2),
                "ms_per_step": round(elapsed / steps * 1e3, 4),
                "kernel_ms": round(kms, 4), "achieved_GBps": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "rccl_gather_ms": (round(gather_ms, 4) if world > 1 and not native else
                                   ("inside dips_diff_series_sharded" if native else 0.0)),
                "step_minus_kernel_ms": round(elapsed / steps * 1e3 - kms, 4),
                "rccl_reference_ms": round(ref_ms, 4) if world > 1 else 0.0,
                "kernel": _v2_kernel_name(mode == Mode.PerFrame, tau),
                "check": chk}
    finally:
        op.close()


def _per_frame_call(torch, n_timed: int, warm: int = 8):
    """The reference's own per-frame pattern (dips/src/frame_extractor.rs:
    206-276 -> lib.rs:233-246 -> gpu/mod.rs:170-397): one 4K RGBA8 frame per
    dips_frame_callback from pageable host memory, the output in host memory
    when the call returns, DiPsProperties defaults (lib.rs:74-86).  Every
    output is compared with the device batch path (frame_callback_batch over
    the same frames in HBM; that path is oracle-tested), outside the timed
    calls.  Returns the record and a small sample for the CPU baseline."""
    from dips_amd import ChromaFilter, ComputeState, DiffSeriesOperator, DiPsFilter, PixelFormat
    W, H = 3840, 2160
    n = warm + n_timed
    props = (False, 1, 5.0, DiPsFilter.Unfiltered, ChromaFilter.None_)
    gen = DiffSeriesOperator(PixelFormat.RGBA8)
    try:
        dev = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
        gen.synth_device(dev, W, H, SEED ^ 0x4A, 0)
    finally:
        gen.close()
    host = dev.cpu().numpy()
    batch = ComputeState(*props)
    try:
        out_dev = torch.empty_like(dev)
        batch.frame_callback_batch_device(dev, out_dev)
        torch.cuda.synchronize()
        want = out_dev.cpu().numpy()
        del out_dev
    finally:
        batch.close()
    del dev
    torch.cuda.empty_cache()
    cs = ComputeState(*props)
    lib, hd = cs._hd._lib, cs._hd
    # every call writes its own output buffer (a caller's ring of frames),
    # faulted in before the timed calls; all outputs are compared after the
    # loop (a compare between calls measured 0.85-0.9x in round 4)
    outs = np.empty_like(host)
    outs.fill(0)
    times, phases = [], []
    cg0, tw0 = {}, 0.0
    try:
        for t in range(n):
            if t == warm:
                cg0, tw0 = _cgroup_cpu_stat(), time.perf_counter()
            t0 = time.perf_counter()
            hd.check(lib.dips_frame_callback(hd.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                             outs[t].ctypes.data, outs[t].nbytes))
            dt = time.perf_counter() - t0
            if t >= warm:
                times.append(dt)
                phases.append(cs.callback_phases())  # outside the timed call
    finally:
        cs.close()
    cg1, tw1 = _cgroup_cpu_stat(), time.perf_counter()
    equal = bool(np.array_equal(outs, want))
    del outs
    fb = W * H * 4
    tot = float(np.sum(times))
    ph = [p for p in phases if p]
    med = lambda k: round(float(np.median([p[k] for p in ph])) / 1e3, 4) if ph else None  # noqa: E731
    breakdown = {
        "phases_ms_median": {
            "sync": med("sync_us"), "staged": med("staged_us"), "launched": med("launched_us"),
            "expand_start": med("expand_start_us"), "last_kernel_wait_end": med("kernels_us"),
            "wall_in_library": med("wall_us")},
        "cpu_ms_per_call_median": {"pack": med("pack_cpu_us"), "expand": med("expand_cpu_us"),
                                   "wait_for_kernels": med("wait_cpu_us")},
        "pool_threads": int(ph[0]["threads"]) if ph else None,
        "cgroup_cpu": ({"cpus_busy_avg": round((cg1["usage_usec"] - cg0["usage_usec"]) / 1e6 / (tw1 - tw0), 2),
                        "throttled_ms": round((cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0)) / 1e3, 2),
                        "nr_throttled": cg1.get("nr_throttled", 0) - cg0.get("nr_throttled", 0),
                        "source": "/sys/fs/cgroup/cpu.stat over the timed calls (the whole process: copy pool + "
                                  "the calling thread + any other thread)"}
                       if cg0 and cg1 and "usage_usec" in cg0 else None),
        "stripes": int(ph[0]["stripes"]) if ph else None,
        "host": _host_cpu(),
        "cpu_bound": {"cpu_ms_per_call_over_threads": (round((med("pack_cpu_us") + med("expand_cpu_us"))
                                                              / int(ph[0]["threads"]), 4) if ph else None),
                      "host_bytes_per_call": 2 * W * H * 4 + W * H * 3,
                      "note": "the pool's pack + expand work spread over its threads, against wall_in_library: the "
                              "CPU side (host memory traffic: the RGBA8 frame read, 2 B/px packed, 1 B/px keys "
                              "read, the RGBA8 output written) bounds the call; the GPU side alone moves a "
                              "frame's packed input and keys in 0.31-0.34 ms (tools/zc_probe.hip)"},
        "note": "phase times from the call's start (dips_callback_phases): staged = last input piece packed "
                "into pinned memory, launched = last stripe kernel launched, expand_start = first output task "
                "started (the pool runs every staging task first), last_kernel_wait_end = last output task past "
                "its wait for its stripe's kernel, wall_in_library = return; cpu sums over the copy pool's tasks",
    } if ph else {"phases": "not recorded (call did not take the zero-copy path)"}
    # the same calls on the all-GPU form (DIPS_FLAG_CROSSCHECK): the whole
    # RGBA8 frame copied into pinned staging and DMA'd to HBM, every step of
    # get_intensity / median / epilogue on the GPU, the RGBA8 output DMA'd
    # back -- no arithmetic on the host
    n_x = min(n_timed, 60)
    cx = ComputeState(*props, crosscheck=True)
    outs_x = np.empty_like(host[:warm + n_x])
    outs_x.fill(0)
    times_x = []
    try:
        lx, hx = cx._hd._lib, cx._hd
        for t in range(warm + n_x):
            t0 = time.perf_counter()
            hx.check(lx.dips_frame_callback(hx.ptr, W, H, host[t].ctypes.data, host[t].nbytes,
                                            outs_x[t].ctypes.data, outs_x[t].nbytes))
            if t >= warm:
                times_x.append(time.perf_counter() - t0)
    finally:
        cx.close()
    all_gpu = {"frames_per_s": round(n_x / float(np.sum(times_x)), 1), "calls": n_x,
               "ms_per_call_median": round(float(np.median(times_x)) * 1e3, 4),
               "outputs_equal_batch_path": bool(np.array_equal(outs_x, want[:warm + n_x])),
               "path": "DIPS_FLAG_CROSSCHECK: add_texture + dispatch with whole-frame RGBA8 DMA both ways "
                       "through pinned staging; get_intensity, the median and the epilogue all on the GPU "
                       "(no host arithmetic); same calls, same frames, same outputs"}
    del outs_x
    rec = {"frames_per_s": round(n_timed / tot, 1), "calls": n_timed,
           "ms_per_call_median": round(float(np.median(times)) * 1e3, 4),
           "ms_per_call_p90": round(float(np.percentile(times, 90)) * 1e3, 4),
           "host_to_device_GBps": round(n_timed * W * H * 2 / tot / 1e9, 2),
           "device_to_host_GBps": round(n_timed * W * H / tot / 1e9, 2),
           "rgba8_GBps_each_way": round(n_timed * fb / tot / 1e9, 2),
           "outputs_equal_batch_path": equal,
           "workload": "3840x2160 RGBA8, DiPsProperties defaults (Unfiltered, window 1, no colour); "
                       f"{warm} untimed calls, then {n_timed} timed dips_frame_callback calls from pageable "
                       "host memory, each into its own pre-faulted pageable output buffer",
           "path": "zero-copy stripes: the copy pool packs each row stripe into pinned memory as what "
                   "get_intensity reads ((max, min) of R, G, B: 2 B/px), and launches "
                   "compat_main_host_packed_kernel on it (PCIe reads of the packed stripe, 1-B gray keys "
                   "written back over PCIe); the pool expands the keys into the RGBA8 output as each stripe's "
                   "event fires (dips_abi.hip frame_callback_striped, copy_pool.h pack_frame / expand_keys)",
           "pcie_bytes_each_way_per_frame": {"host_to_device": W * H * 2, "device_to_host": W * H},
           "all_gpu_form": all_gpu,
           "breakdown": breakdown}
    return rec, (host[:warm].copy(), want[:warm].copy())


# identity of this rank for failure reports: rank, local device, PCI bus id
_WHO = {"rank": os.environ.get("RANK", "0"), "local": os.environ.get("LOCAL_RANK", "0"), "bus": None}


# The JSON line goes to the process's real stdout; everything else written to
# fd 1 -- RCCL prints its version banner there when a communicator is made --
# goes to stderr, so that rank 0's stdout holds the one line and nothing else.
_LINE_FD = None


def _stdout_for_the_line_only():
    global _LINE_FD
    sys.stdout.flush()
    _LINE_FD = os.dup(1)
    os.dup2(2, 1)


def _emit_line(text: str) -> None:
    os.write(_LINE_FD if _LINE_FD is not None else 1, (text + "\n").encode())


def main():
    """Run the bench; any exception on any rank ends THIS process with a
    non-zero status after naming the rank and its device's PCI bus id (a rank
    left waiting in a collective fails at the process group's timeout,
    --dist-timeout, instead of hanging until the driver's limit)."""
    args = parse()
    _stdout_for_the_line_only()
    try:
        _main(args)
    except SystemExit:
        raise
    except BaseException:
        log(f"FAILED on rank {_WHO['rank']} (local device {_WHO['local']}, PCI {_WHO['bus']}):\n"
            f"{traceback.format_exc()}")
        sys.stdout.flush()
        sys.stderr.flush()
        # no destructors: a process group or a HIP context in a failed state
        # can block in its teardown
        os._exit(1)


def _main(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    # Rehearsal of the N > 1 path on one GPU (tests/test_gpu_bench_rehearsal.py):
    # DIPS_BENCH_BACKEND=gloo with DIPS_BENCH_ONE_DEVICE=1 runs every rank on
    # device 0 over gloo, which on this torch build moves device tensors for
    # every collective the step uses (tools/gloo_cuda_probe.py).  The line then
    # says so in "parallelism"; the driver's runs use RCCL, one rank per GPU.
    backend = os.environ.get("DIPS_BENCH_BACKEND", "nccl")
    if os.environ.get("DIPS_BENCH_ONE_DEVICE") == "1":
        local = 0
    corrupt_halo = os.environ.get("DIPS_BENCH_CORRUPT_HALO") == "1"  # the self-check must catch it (tests)
    torch.cuda.set_device(local)  # one rank per GPU (RCCL rejects two ranks on one device)
    _WHO["local"] = local
    try:
        pr = torch.cuda.get_device_properties(local)
        _WHO["bus"] = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    except Exception:  # the report only
        pass
    # N > 1: the native sharded call (default) or the torch protocol.  Neither
    # caps the series grid for the halo's kernels: posted first, they run
    # beside the full grid at +0.03-0.07 ms, where a grid one wave per SIMD
    # short cost 2-5 ms (profiles/r06/halo_contention/)
    shard_path = os.environ.get("DIPS_BENCH_SHARD", "native") if world > 1 else None
    dev = torch.device("cuda", local)
    if world > 1:
        # a bounded wait: a rank stuck in a collective (a peer that died, a
        # lost RCCL connection) fails after --dist-timeout seconds
        tmo = timedelta(seconds=args.dist_timeout)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        log(f"rank {rank}/{world}: device {local} PCI {_WHO['bus']}, backend {backend}")
    if os.environ.get("DIPS_BENCH_FAIL_RANK") == str(rank):  # the failure report path (tests)
        raise RuntimeError("DIPS_BENCH_FAIL_RANK: injected failure")

    from dips_amd import DiffSeriesOperator, Mode, PixelFormat, shard

    # the native sharded path's communicator: RCCL (driver runs) or the host
    # transport over gloo (the one-GPU rehearsal); every rank must get one,
    # else all fall back to the torch protocol and the line says why
    comm, comm_note = None, None
    if shard_path == "native":
        comm, comm_note = _make_comm(torch, dist, backend, world, rank, local, corrupt_halo)
        if comm is None:
            shard_path = "torch"

    W, H, F = args.width, args.height, args.frames_per_gpu
    C = 3
    fb = W * H * C
    mode = Mode.PerFrame if args.mode == "per-frame" else Mode.Overall
    op = DiffSeriesOperator(PixelFormat.RGB8, mode, args.tau, time_kernel=True, device=local)

    t0 = rank * F  # global frame index of this rank's first frame
    # the batch in the plain allocation, or in a second candidate placement
    # when that runs faster by > 1 % (where the driver puts a 124 GB buffer
    # moves this power-bound kernel by 2-3 points; tools/placement.py), both
    # candidates' times reported in the line
    from tools.placement import resident_frames
    frames, placement = resident_frames(
        op, (F, H, W, C), dev, lambda t: op.synth_device(t, W, H, SEED, t0),
        probe=not args.no_placement_probe, ref_of=(lambda t: t[0]) if mode == Mode.Overall else None)
    series = torch.zeros((F, 4), dtype=torch.int64, device=dev)
    ref = torch.empty((H, W, C), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    log(f"rank {rank}: {F} frames {W}x{H} RGB8 = {F * fb / 1e9:.1f} GB generated in HBM")

    # Reference frame of the rank's first frame ('overall': broadcast once per
    # job, the reference is fixed; 'per-frame': the halo frame, exchanged
    # every step -- inside dips_diff_series_sharded on the native path, by
    # dips_amd.shard.per_frame_overlapped on the torch path).
    if mode == Mode.Overall:
        if comm is not None:
            op.shard_broadcast_device(comm, frames[0] if rank == 0 else None, ref)
            torch.cuda.synchronize()
        else:
            if rank == 0:
                ref.copy_(frames[0])
            shard.broadcast_reference(ref, src=0)
    if comm is not None:
        gathered = torch.zeros((world * F, 4), dtype=torch.int64, device=dev) if rank == 0 else None

        def step():
            # halo send/recv beside the series launch, one ncclGather
            op.run_sharded(comm, frames, world * F, series, gathered,
                           ref=ref if mode == Mode.Overall else None, ref_resident=mode == Mode.Overall)
            return gathered
    else:
        gather = shard.SeriesGather(world * F, dev)

        def compute(fr, r, out):
            if corrupt_halo and rank == 1 and r is ref:
                r.view(-1)[12345] ^= 0x5A  # the received halo frame, damaged on purpose
            op.run_device(fr, out, ref=r)

        def step():
            if mode == Mode.Overall:
                compute(frames, ref, series)
            elif world == 1:
                compute(frames, None, series)
            else:
                # the halo transfer overlaps the compute of frames 1..F-1
                shard.per_frame_overlapped(frames, ref, series, compute)
            return gather(series)

    smp = _power_sampler(torch, local) if rank == 0 else None
    final = None
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    op.kernel_time(reset=True)

    def timed_steps():
        # barrier + synchronize on both sides (rank 0's power reading before
        # this is outside every rank's clock)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = None
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        return out, time.perf_counter() - t

    (final, elapsed), power = _power_leg(smp, timed_steps, F * args.steps, "the timed steps")
    kms, launches = op.kernel_time()
    each = op.kernel_times()  # one launch per step at N = 1 (two at N > 1 per-frame)
    # measured read-only ceilings on this GPU, outside the timed region, each
    # as many back-to-back launches as the timed steps ran, between power
    # readings of its own (does the gap to the ceiling coincide with
    # throttling the ceiling does not see?): one plain stream over the same
    # resident bytes, and the series kernel's own access shape (tile walk,
    # schedule, 12-B vecs, no compute)
    reps = max(3, args.steps)
    read_all, read_power = _power_leg(smp, lambda: [op.read_ceiling_ms(frames) for _ in range(reps)], F * reps,
                                      f"{reps} back-to-back read_ceiling_kernel launches")
    walk_all, walk_power = _power_leg(smp, lambda: [op.read_ceiling_walk_ms(frames) for _ in range(reps)],
                                      F * reps, f"{reps} back-to-back read_walk_kernel launches")
    read_ms, walk_ms = float(np.median(read_all)), float(np.median(walk_all))
    # series-kernel time per step (one launch per step, two when the halo
    # overlap splits a per-frame batch at N > 1)
    tt = torch.tensor([elapsed, kms / args.steps], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed_max, kernel_ms = float(tt[0]), float(tt[1])

    devices = _devices(torch, dist, world, local)
    placements = _gather_objects(dist, world, placement)
    # Self-check of the timed step at every world size (collective): each
    # rank re-derives its first entries against the halo / reference it
    # received, rank 0 re-derives the gathered rows at every shard boundary
    # and 8 random frames (dips_amd.shard.verify_sharded_series)
    check = None
    if comm is not None and mode == Mode.PerFrame and world > 1:
        # what the library compared this rank's first frame with: the halo it
        # received (rank > 0), for the self-check below
        op.shard_reference_device(ref)
        torch.cuda.synchronize()
    if not args.no_check:
        check = shard.verify_sharded_series(op, width=W, height=H, seed=SEED, n_total=world * F,
                                            per_frame=(mode == Mode.PerFrame), local_series=series, ref=ref,
                                            gathered=final, device=dev)
        picks = check.pop("global_frames")
        log(f"check: {check['frames_checked']} frames re-derived (global {picks[:12]}...), equal={check['equal']}")
    waves, tiles, pbytes = op.geometry(W, H, F)
    algo_bytes = F * fb  # each frame read once per launch
    achieved = algo_bytes / (kernel_ms / 1e3) / 1e9
    value = world * F * args.steps / elapsed_max

    pcie = mapv = cpu = pfc = tau0 = None
    if rank == 0:
        final_np = final.cpu().numpy().view(np.uint64)
        assert final_np.shape == (world * F, 4)
        if args.dump_series:
            np.save(args.dump_series, final_np)
        if args.check and world * F * fb > (64 << 30):
            log("--check skipped: the N*F frames would not fit beside the resident batch (small sizes only)")
        elif args.check:
            # the same N*F frames in one launch on one device (small sizes only)
            allf = torch.empty((world * F, H, W, C), dtype=torch.uint8, device=dev)
            op.synth_device(allf, W, H, SEED, 0)
            one = torch.zeros((world * F, 4), dtype=torch.int64, device=dev)
            op.run_device(allf, one, ref=None if mode == Mode.PerFrame else allf[0])
            torch.cuda.synchronize()
            assert np.array_equal(final_np, one.cpu().numpy().view(np.uint64)), "gathered series != single-device series"
            log(f"--check: gathered series of {world}x{F} frames equals the single-device series")
            del allf, one
    if world == 1:
        # PCIe-inclusive rate, reported beside (never as) `value` (BASELINE.md:
        # "the H2D end-to-end rate separately"): the first 96 frames copied to
        # pageable host memory and fed back through dips_diff_series_streamed
        try:
            if args.no_pcie:
                raise RuntimeError("--no-pcie")
            nh = min(F, 96)
            host = frames[:nh].cpu().numpy()
            op.streamed(host[:16], chunk_frames=8)  # warm (pinned / ring allocations)
            t_h = time.perf_counter()
            sh = op.streamed(host, chunk_frames=8)
            dt_h = time.perf_counter() - t_h
            want = series[:nh].cpu().numpy().view(np.uint64)
            pcie = {"frames_per_s": round(nh / dt_h, 1), "host_to_device_GBps": round(nh * fb / dt_h / 1e9, 2),
                    "frames": nh, "path": "pageable host frames -> pooled pinned staging -> H2D on a side "
                                          "stream, series kernel on the previous chunk (dips_diff_series_streamed)",
                    "series_matches_resident_run": bool(np.array_equal(sh.as_array(), want))}
            del host
        except Exception as e:  # report, never hide
            pcie = {"skipped": str(e)}
        if not args.no_tau0:
            try:
                tau0 = _tau0_leg(torch, smp, DiffSeriesOperator, frames, series, mode == Mode.PerFrame, args.tau,
                                 max(3, args.steps), device=local)
                log(f"tau0: frac {tau0['frac']}, power {tau0['power']}")
            except Exception as e:  # report, never hide
                tau0 = {"skipped": str(e)}
        if not args.no_map:
            try:
                mapv = _map_variant(torch, DiffSeriesOperator, frames, min(F, args.map_frames), W, H,
                                    mode == Mode.PerFrame, args.tau)
            except Exception as e:  # report, never hide
                mapv = {"skipped": str(e)}
        pf_sample = None
        if not args.no_per_frame_call:
            try:
                pfc, pf_sample = _per_frame_call(torch, args.per_frame_calls)
                log(f"per_frame_call: {pfc['frames_per_s']} frames/s, outputs equal: {pfc['outputs_equal_batch_path']}")
            except Exception as e:  # report, never hide
                pfc = {"skipped": str(e)}
        if not args.no_cpu_baseline:
            try:
                cpu = cpu_baseline(frames, series, int(mode), args.tau, args.cpu_seconds,
                                   op_gray=lambda fr, want: _config0_gpu(torch, fr, want), pf_sample=pf_sample)
            except Exception as e:  # report, never hide
                cpu = {"value": None, "unit": "frames/s", "cores": 0, "kind": "port",
                       "sample": f"failed: {e}"}
            pf_sample = None

    # configs[3] and configs[4] on the same ranks, regenerated into the same
    # resident buffer (collective at N > 1)
    legs = {}
    if not args.no_legs:
        op.close()
        op = None
        del series
        buf = frames
        del frames
        W8, H8 = 2 * W, 2 * H
        for key, name, lw, lh, lf in (
                ("configs3", "BASELINE.json configs[3]: 3840x2160 RGB8, 'overall', reference broadcast, "
                             f"{F} frames per GPU", W, H, F),
                ("configs4", "BASELINE.json configs[4]: 7680x4320 RGB8, 'overall', f32 intensity with threshold "
                             f"tau={args.tau:.6g}, {(F * fb) // (W8 * H8 * 3)} frames per GPU", W8, H8,
                 (F * fb) // (W8 * H8 * 3))):
            try:
                if lf < 2:
                    raise ValueError("fewer than 2 frames per GPU at this size")
                legs[key] = _config_leg(torch, dist, buf, name=name, W=lw, H=lh, F=lf, mode=Mode.Overall,
                                        tau=args.tau, steps=args.leg_steps, world=world, rank=rank, local=local,
                                        dev=dev, check=not args.no_check, comm=comm,
                                        dump=(os.path.splitext(args.dump_series)[0] + f"_{key}.npy"
                                              if args.dump_series else None))
                log(f"{key}: {legs[key]['frames_per_s']} frames/s, frac {legs[key]['frac']}, "
                    f"check {legs[key]['check']}")
            except Exception as e:  # report, never hide
                legs[key] = {"failed": f"{type(e).__name__}: {e}"}
        del buf

    ok = all(c is None or c.get("equal") for c in [check] + [l.get("check") for l in legs.values()])
    ok = ok and all("failed" not in l for l in legs.values())
    if rank == 0:
        traffic = None
        pmc_note = None
        lib_sha = _lib_sha256()
        if os.path.exists(args.pmc_json):
            try:
                with open(args.pmc_json) as f:
                    pmc = json.load(f)
                same_run = (pmc.get("width"), pmc.get("height"), pmc.get("frames"), pmc.get("mode")) == (W, H, F, args.mode)
                if same_run and pmc.get("lib_sha256") == lib_sha:
                    traffic = pmc.get("hbm_bytes_per_launch")
                    pmc_note = pmc.get("source")
                else:
                    pmc_note = ("traffic null: profiles/pmc_traffic.json was collected with another build of "
                                "libdips_hip.so or another workload")
            except Exception:
                traffic = None
        out = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (shared integer-hash generator, frames generated in HBM)",
            "config": {
                "workload": f"{W}x{H} RGB8, {F} frames per GPU, '{args.mode}' mode, tau={args.tau:.6g} "
                            f"(BASELINE.json configs[{2 if mode == Mode.PerFrame else 3}] per-GPU slice)",
                "frames_per_gpu": F, "width": W, "height": H, "mode": args.mode,
                "parallelism": f"frame-range x{world}" + (
                    ((" native dips_diff_series_sharded: RCCL halo ncclSend/ncclRecv beside the series launch "
                      "+ one ncclGather" if backend == "nccl" else
                      f" native dips_diff_series_sharded over the {backend} host transport (rehearsal, ranks "
                      "share one GPU)") if shard_path == "native" else
                     (" + RCCL halo send/recv + gather (torch protocol, dips_amd.shard)" if backend == "nccl"
                      else f" + {backend} halo send/recv + gather (torch protocol; rehearsal, ranks share one "
                           "GPU)")) if world > 1 else ""),
            },
            "shard_path": ({"path": shard_path, **(comm_note or {})} if world > 1 else None),
            "ranks": world,
            "devices": devices,
            "placement": placements,
            "check": check,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": _v2_kernel_name(mode == Mode.PerFrame, args.tau),
                "kernel_ms": round(kernel_ms, 4),
                "kernel_ms_median": round(float(np.median(each)), 4) if world == 1 and each else None,
                "kernel_launches_timed": len(each),
                # what a plain caller gets: the batch's first allocation
                # (tools/placement.py candidate 0, the median of its probe
                # launches), beside the headline's kept placement
                **_plain_allocation(placement, algo_bytes, kernel_ms),
                "read_ceiling": {
                    "achieved": round(F * fb / (read_ms / 1e3) / 1e9, 1),
                    "unit": "GB/s",
                    "frac": round(achieved / (F * fb / (read_ms / 1e3) / 1e9), 4),
                    "kernel": "read_ceiling_kernel: non-temporal 16-B loads, 4 in flight per lane, grid-stride, "
                              "over the same frames (no compute)",
                    "launches": len(read_all),
                    "power": read_power,
                    "series_shape": {
                        "achieved": round(F * fb / (walk_ms / 1e3) / 1e9, 1),
                        "frac": round(achieved / (F * fb / (walk_ms / 1e3) / 1e9), 4),
                        "kernel": "read_walk_kernel: the series kernel's tile walk, schedule (part-major for "
                                  "batches of >= 256 frames, either mode) and vecs over the same frames, no compute",
                        "launches": len(walk_all),
                        "power": walk_power,
                    },
                },
                "algorithmic_bytes_per_launch": algo_bytes,
                "partial_bytes_per_launch": int(pbytes) * F,
                "waves": int(waves),
                **({"traffic_source": pmc_note} if pmc_note else {}),
                "lib_sha256": lib_sha,
            },
            "cpu_baseline": cpu,
            "power": power,
            "tau0": tau0,
            "pcie_inclusive": pcie,
            "map_variant": mapv,
            "per_frame_call": pfc,
            **legs,
        }
        _emit_line(json.dumps(out))
    if op is not None:
        op.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        log("FAILED: a self-check of the sharded series did not match (see 'check' in the JSON line)")
        sys.exit(1)


if __name__ == "__main__":
    main()
