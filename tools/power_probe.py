#!/usr/bin/env python3
"""power_probe.py -- socket power, energy and shader clock of the series path
under sustained load (read-only queries through the amdsmi library; nothing
is changed on the device).

Why: the series kernel runs at ~1.56 GHz while streaming and ~2.07 GHz
compute-only (GRBM_GUI_ACTIVE), which reads as a power-limited
clock.  This measures it directly: each phase runs one workload back to back
for a few seconds over the same 5000 resident 4K RGB8 frames while a thread
samples the energy accumulator, the socket power and the per-XCD gfx clocks.

Phases: idle; series_v2_kernel (per-frame, tau 8/255: the headline);
the read-only walk of the same access shape (dips_read_ceiling_walk); the
grid-stride read (dips_read_ceiling); the compute-only build of the series
kernel (build/probe_same: every wave re-reads one frame from L2, run as a
child process over 1000 frames).  Output: one JSON line per phase (rate,
average power from the energy counter, mean clock, energy per frame) to
stdout.

Run on the GPU box:  python tools/power_probe.py [seconds_per_phase]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W, H, C, F = 3840, 2160, 3, 5000
FB = W * H * C


class Sampler(threading.Thread):
    """Polls every GPU handle amdsmi reports: (t, energy J, socket W, clocks)."""

    def __init__(self, period=0.02, pci_bus=None):
        super().__init__(daemon=True)
        import amdsmi
        self.smi = amdsmi
        amdsmi.amdsmi_init()
        self.handles = amdsmi.amdsmi_get_processor_handles()
        if pci_bus is not None:
            # only the GPU on this PCI bus (bench.py: the rank's own device)
            keep = []
            for h in self.handles:
                try:
                    bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)
                    if int(bdf.split(":")[1], 16) == int(pci_bus):
                        keep.append(h)
                except Exception:  # noqa: BLE001
                    pass
            self.handles = keep
        self.period = period
        self.rows = []  # (t, handle index, energy_J, socket_W, mean gfxclk MHz, hotspot C, throttle)
        self.stop_ev = threading.Event()
        self.info = []
        for h in self.handles:
            d = {}
            try:
                d["bdf"] = amdsmi.amdsmi_get_gpu_device_bdf(h)
            except Exception as e:  # noqa: BLE001
                d["bdf"] = str(e)
            try:
                d["power_cap"] = amdsmi.amdsmi_get_power_cap_info(h)
            except Exception as e:  # noqa: BLE001
                d["power_cap"] = str(e)
            self.info.append(d)

    RES = ("accumulation_counter", "prochot_residency_acc", "ppt_residency_acc", "socket_thm_residency_acc",
           "vr_thm_residency_acc", "hbm_thm_residency_acc")

    def sample(self):
        smi = self.smi
        t = time.monotonic()
        for k, h in enumerate(self.handles):
            try:
                e = smi.amdsmi_get_energy_count(h)
                ej = e["energy_accumulator"] * e["counter_resolution"] * 1e-6
            except Exception:  # noqa: BLE001
                ej = None
            extra = {}
            try:
                m = smi.amdsmi_get_gpu_metrics_info(h)
                clks = [c for c in (m.get("current_gfxclks") or []) if isinstance(c, int) and c > 0]
                clk = float(np.mean(clks)) if clks else None
                pw = m.get("current_socket_power")
                pw = pw if isinstance(pw, (int, float)) else None
                hot = m.get("temperature_hotspot")
                hot = hot if isinstance(hot, (int, float)) else None
                thr = m.get("indep_throttle_status")
                for key in self.RES + ("voltage_gfx", "current_uclk", "average_umc_activity", "temperature_hbm"):
                    extra[key] = m.get(key)
            except Exception:  # noqa: BLE001
                clk = pw = hot = thr = None
            self.rows.append((t, k, ej, pw, clk, hot, thr, extra))

    def run(self):
        while not self.stop_ev.is_set():
            self.sample()
            time.sleep(self.period)

    def _residency(self, rs):
        """Fraction of the window each throttler was active (residency
        accumulators over the accumulation counter), gfx voltage, uclk."""
        out = {}
        a, b = rs[0][7], rs[-1][7]
        try:
            dn = b["accumulation_counter"] - a["accumulation_counter"]
            if dn > 0:
                for key in self.RES[1:]:
                    out[key.replace("_acc", "_frac")] = round((b[key] - a[key]) / dn, 4)
        except (TypeError, KeyError):
            pass
        for key in ("voltage_gfx", "current_uclk", "average_umc_activity", "temperature_hbm"):
            v = [r[7].get(key) for r in rs if isinstance(r[7].get(key), (int, float))]
            if v:
                out[key + "_mean"] = round(float(np.mean(v)), 1)
        return out

    def window(self, t0, t1):
        """Per handle: average power from the energy counter over [t0, t1],
        mean sampled socket power, mean clock, max hotspot."""
        out = []
        for k in range(len(self.handles)):
            rs = [r for r in self.rows if r[1] == k and t0 <= r[0] <= t1]
            if len(rs) < 2:
                out.append(None)
                continue
            e = [r for r in rs if r[2] is not None]
            p_e = (e[-1][2] - e[0][2]) / (e[-1][0] - e[0][0]) if len(e) >= 2 and e[-1][0] > e[0][0] else None
            pw = [r[3] for r in rs if r[3] is not None]
            ck = [r[4] for r in rs if r[4] is not None]
            hot = [r[5] for r in rs if r[5] is not None]
            out.append({"handle": k, "avg_power_W_energy": round(p_e, 1) if p_e is not None else None,
                        "socket_power_W_mean": round(float(np.mean(pw)), 1) if pw else None,
                        "gfxclk_MHz_mean": round(float(np.mean(ck)), 1) if ck else None,
                        "gfxclk_MHz_min": round(float(np.min(ck)), 1) if ck else None,
                        "hotspot_C_max": max(hot) if hot else None, "samples": len(rs),
                        "indep_throttle_status": sorted({str(r[6]) for r in rs}),
                        **self._residency(rs)})
        return out


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 6.0
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat

    smp = Sampler()
    smp.start()
    print(json.dumps({"handles": smp.info}), flush=True)
    if os.environ.get("POWER_PROBE_GRAY") == "1":
        return gray_phases(smp, secs)
    if os.environ.get("POWER_PROBE_VISUAL") == "1":
        return visual_phases(smp, secs)
    op = DiffSeriesOperator(PixelFormat.RGB8, Mode.PerFrame, 8.0 / 255.0, time_kernel=True)
    frames = torch.empty((F, H, W, C), dtype=torch.uint8, device="cuda")
    op.synth_device(frames, W, H, 0xD1B5, 0)
    series = torch.zeros((F, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def report(name, t0, t1, launches, frames_per_launch, extra=None):
        dt = t1 - t0
        fps = launches * frames_per_launch / dt
        per = smp.window(t0 + 0.25 * dt, t1)  # skip the ramp
        main_h = max((p for p in per if p), key=lambda p: p["avg_power_W_energy"] or 0.0, default=None)
        row = {"phase": name, "seconds": round(dt, 2), "launches": launches, "frames_per_s": round(fps, 1),
               "GBps": round(fps * FB / 1e9, 1), "frac_of_8TBps": round(fps * FB / 1e9 / 8000.0, 4),
               "gpu": main_h}
        if main_h and main_h.get("avg_power_W_energy") and fps > 0:
            row["joules_per_frame"] = round(main_h["avg_power_W_energy"] / fps, 5)
        if extra:
            row.update(extra)
        print(json.dumps(row), flush=True)

    # idle
    t0 = time.monotonic()
    time.sleep(min(2.0, secs))
    report("idle", t0, time.monotonic(), 0, 0)

    # the headline kernel, back to back (default 5 waves per SIMD, then
    # capped at 4 and 3 through DIPS_SERIES_WAVES_PER_SIMD, read per launch)
    waves = [w for w in os.environ.get("POWER_PROBE_WAVES", "0,4,3").split(",") if w]
    for wv in waves:
        if wv == "0":
            os.environ.pop("DIPS_SERIES_WAVES_PER_SIMD", None)
        else:
            os.environ["DIPS_SERIES_WAVES_PER_SIMD"] = wv
        op.run_device(frames, series)
        torch.cuda.synchronize()
        op.kernel_time(reset=True)
        n, t0 = 0, time.monotonic()
        while time.monotonic() - t0 < secs:
            for _ in range(10):
                op.run_device(frames, series)
            torch.cuda.synchronize()
            n += 10
        t1 = time.monotonic()
        each = op.kernel_times()
        report(f"series_v2_kernel<3,0,4,PF=true> (headline), waves/SIMD {'default' if wv == '0' else wv}",
               t0, t1, n, F,
               {"kernel_ms_median": round(float(np.median(each)), 3),
                "kernel_ms_first_last10": [round(float(np.mean(each[:10])), 3),
                                           round(float(np.mean(each[-10:])), 3)]})
    os.environ.pop("DIPS_SERIES_WAVES_PER_SIMD", None)

    # read-only walk of the same access shape, and the grid-stride read
    for name, fn in (("read walk (series access shape, no compute)", op.read_ceiling_walk_ms),
                     ("grid-stride read (16-B nt loads)", lambda fr: op.read_ceiling_ms(fr))):
        n, t0, ms = 0, time.monotonic(), []
        while time.monotonic() - t0 < secs:
            ms.append(fn(frames))
            n += 1
        report(name, t0, time.monotonic(), n, F, {"kernel_ms_median": round(float(np.median(ms)), 3)})

    del frames, series
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    op.close()

    # compute-only build (child process; its 1000 frames are generated
    # first, so the window starts after a short ramp)
    exe = os.path.join(ROOT, "build", "probe_same")
    if os.path.exists(exe):
        rounds = max(50, int(secs / 0.0036))
        t0 = time.monotonic()
        r = subprocess.run([exe, "1000", str(rounds), "v2<U=kUnrollV2,PF=true> tau=8.0f"], capture_output=True,
                           text=True, timeout=600)
        t1 = time.monotonic()
        line = [l for l in r.stdout.splitlines() if "median" in l]
        med = None
        if line:
            try:
                med = float(line[-1].split("median")[1].split("ms")[0])
            except (IndexError, ValueError):
                med = None
        # launches = rounds (+1 parity run); frames/s from the median launch
        dt = t1 - t0
        per = smp.window(t0 + 0.3 * dt, t1 - 0.05 * dt)
        main_h = max((p for p in per if p), key=lambda p: p["avg_power_W_energy"] or 0.0, default=None)
        fps = 1000.0 / (med / 1e3) if med else None
        row = {"phase": "series_v2_kernel compute-only (build/probe_same: every wave re-reads one frame)",
               "seconds": round(dt, 2), "launches": rounds, "kernel_ms_median": med,
               "frames_per_s": round(fps, 1) if fps else None, "gpu": main_h, "rc": r.returncode,
               "probe_line": line[-1] if line else r.stderr[-300:]}
        if main_h and main_h.get("avg_power_W_energy") and fps:
            row["joules_per_frame"] = round(main_h["avg_power_W_energy"] / fps, 5)
        print(json.dumps(row), flush=True)
    smp.stop_ev.set()
    smp.join(timeout=2)


def gray_phases(smp, secs):
    """4K GRAY8 per-frame (the LDS-table kernel, 15,000 resident frames) and
    the grid-stride read of the same bytes."""
    import torch
    from dips_amd import DiffSeriesOperator, Mode, PixelFormat
    n = 15000
    fb = W * H
    op = DiffSeriesOperator(PixelFormat.Gray8, Mode.PerFrame, 8.0 / 255.0, time_kernel=True)
    frames = torch.empty((n, H, W), dtype=torch.uint8, device="cuda")
    op.synth_device(frames, W, H, 0xD1B5, 0)
    series = torch.zeros((n, 4), dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def rep(name, t0, t1, launches, extra):
        dt = t1 - t0
        fps = launches * n / dt
        per = smp.window(t0 + 0.25 * dt, t1)
        main_h = max((p for p in per if p), key=lambda p: p["avg_power_W_energy"] or 0.0, default=None)
        row = {"phase": name, "seconds": round(dt, 2), "launches": launches, "frames_per_s": round(fps, 1),
               "GBps": round(fps * fb / 1e9, 1), "frac_of_8TBps": round(fps * fb / 1e9 / 8000.0, 4), "gpu": main_h}
        if main_h and main_h.get("avg_power_W_energy") and fps > 0:
            row["joules_per_frame"] = round(main_h["avg_power_W_energy"] / fps, 6)
        row.update(extra)
        print(json.dumps(row), flush=True)

    op.run_device(frames, series)
    torch.cuda.synchronize()
    op.kernel_time(reset=True)
    k, t0 = 0, time.monotonic()
    while time.monotonic() - t0 < secs:
        for _ in range(10):
            op.run_device(frames, series)
        torch.cuda.synchronize()
        k += 10
    t1 = time.monotonic()
    each = op.kernel_times()
    rep("series_gray_lut_kernel (4K gray8, per-frame)", t0, t1, k,
        {"kernel_ms_median": round(float(np.median(each)), 3)})
    k, t0, ms = 0, time.monotonic(), []
    while time.monotonic() - t0 < secs:
        ms.append(op.read_ceiling_ms(frames))
        k += 1
    rep("grid-stride read (16-B nt loads), gray frames", t0, time.monotonic(), k,
        {"kernel_ms_median": round(float(np.median(ms)), 3)})
    op.close()
    smp.stop_ev.set()
    smp.join(timeout=2)


def visual_phases(smp, secs):
    """The two visual operators over 1000 resident 4K RGBA8 frames, back to
    back: dips ComputeState frame_callback_batch (colour + sigmoid, the (S, m)
    table kernel) and the dips_alt run loop (default properties, the diff
    table kernel); bytes = read + write per frame."""
    import torch
    from dips_amd import DiffSeriesOperator, PixelFormat
    from dips_amd.api import ChromaFilter, ComputeState, DiPsFilter
    from dips_amd.alt import DiPsCompute
    n = 1000
    fb = W * H * 4
    frames = torch.empty((n, H, W, 4), dtype=torch.uint8, device="cuda")
    syn = DiffSeriesOperator(PixelFormat.RGBA8)
    syn.synth_device(frames, W, H, 0xD1B5, 0)
    syn.close()
    out = torch.empty_like(frames)
    torch.cuda.synchronize()

    def rep(name, t0, t1, launches):
        dt = t1 - t0
        fps = launches * n / dt
        g = smp.window(t0 + 0.25 * dt, t1)[0]
        row = {"phase": name, "seconds": round(dt, 2), "launches": launches, "frames_per_s": round(fps, 1),
               "GBps_read_write": round(fps * 2 * fb / 1e9, 1), "frac_of_8TBps": round(fps * 2 * fb / 1e9 / 8000, 4),
               "gpu": g}
        if g and g.get("avg_power_W_energy"):
            row["mJ_per_frame"] = round(g["avg_power_W_energy"] / fps * 1e3, 4)
        print(json.dumps(row), flush=True)

    cs = ComputeState(True, 1, 5.0, DiPsFilter.Sigmoid, ChromaFilter.None_)
    cs.frame_callback_batch_device(frames[:7], out[:7])
    cs.frame_callback_batch_device(frames, out)
    torch.cuda.synchronize()
    k, t0 = 0, time.monotonic()
    while time.monotonic() - t0 < secs:
        for _ in range(5):
            cs.frame_callback_batch_device(frames, out)
        torch.cuda.synchronize()
        k += 5
    rep("compat_batch_lut_kernel (ComputeState batch, colour + sigmoid)", t0, time.monotonic(), k)
    cs.close()
    flags = [t == 2 for t in range(n)]
    c = DiPsCompute(2, H, W)
    c.send_frames_device(frames, out, flags)
    torch.cuda.synchronize()
    k, t0 = 0, time.monotonic()
    while time.monotonic() - t0 < secs:
        for _ in range(5):
            c.send_frames_device(frames, out, flags)
        torch.cuda.synchronize()
        k += 5
    rep("alt_batch_kernel LUT (dips_alt run loop, default properties)", t0, time.monotonic(), k)
    c.close()
    smp.stop_ev.set()
    smp.join(timeout=2)


if __name__ == "__main__":
    main()
