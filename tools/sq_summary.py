#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh: per build (real frames / compute-only), the
last series_v2_kernel dispatch of every pass -> duration, effective shader
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), VALU instructions per SIMD
cycle, wave-cycle fractions waiting / issuing."""
import csv
import glob
import os
import sys

N_XCD, N_SIMD = 8, 1024


def last_dispatch(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "series_v2_kernel" in r["Kernel_Name"]:
                rows.setdefault(int(r["Dispatch_Id"]), []).append(r)
    if not rows:
        return None, {}
    did = max(rows)
    vals = {r["Counter_Name"]: float(r["Counter_Value"]) for r in rows[did]}
    r0 = rows[did][0]
    return (int(r0["End_Timestamp"]) - int(r0["Start_Timestamp"])) * 1e-9, vals


def main():
    root = sys.argv[1]
    print("series_v2_kernel<3,0,4,PF=true,MAP=false>, 1000 4K RGB8 frames (tools/pmc_sq.sh); last dispatch per pass")
    for b, label in (("probe", "real frames"), ("probe_same", "compute-only (one frame re-read)")):
        c, durs = {}, []
        for d in sorted(glob.glob(os.path.join(root, b + ".*"))):
            if not os.path.isdir(d):
                continue
            dur, vals = last_dispatch(d)
            if dur:
                durs.append(dur)
                c.update(vals)
        if not durs:
            print(f"{label}: no data")
            continue
        dur = sum(durs) / len(durs)
        clk = c.get("GRBM_GUI_ACTIVE", 0) / N_XCD / dur
        simd_cycles = clk * dur * N_SIMD
        line = [f"{label}: duration {dur * 1e3:.3f} ms (mean of {len(durs)} passes)",
                f"clock {clk / 1e9:.3f} GHz",
                f"GB/s {1000 * 24883200 / dur / 1e9:.0f}"]
        if "SQ_INSTS_VALU" in c and simd_cycles:
            line.append(f"VALU insts/SIMD-cycle {c['SQ_INSTS_VALU'] / simd_cycles:.3f}")
            line.append(f"SALU/VALU {c.get('SQ_INSTS_SALU', 0) / c['SQ_INSTS_VALU']:.3f}")
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            wc = c["SQ_WAVE_CYCLES"]
            for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in c:
                    line.append(f"{k}/wave-cycle {c[k] / wc:.3f}")
        print(", ".join(line))
        print("  raw: " + ", ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
