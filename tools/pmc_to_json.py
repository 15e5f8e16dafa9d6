"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into the
per-launch HBM traffic of the series kernel (profiles/pmc_traffic.json).

gfx950 corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE reads exactly
half the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact
for streaming stores.  Both are reported in KiB per dispatch."""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def lib_sha256() -> str:
    """sha256 of the library the counters were collected with (bench.py uses
    the traffic only for this very build)."""
    import hashlib
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "dips_amd", "lib", "libdips_hip.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def main():
    # usage: pmc_to_json.py DIR FRAMES MODE OUT [KERNEL BYTES_PER_FRAME]
    d, frames, mode, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    kernel = sys.argv[5] if len(sys.argv) > 5 else "series_v2_kernel"
    W, H = 3840, 2160
    bpf = int(sys.argv[6]) if len(sys.argv) > 6 else W * H * 3
    fetch = per_dispatch(d, "FETCH_SIZE", kernel)
    write = per_dispatch(d, "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} rows (fetch {len(fetch)}, write {len(write)})")
    # the largest dispatches are the timed full-batch launches (a run may also
    # hold short parity-check launches of the same kernel)
    full_f = [v for v in fetch if v >= 0.9 * max(fetch)]
    full_w = [v for v in write if v >= 0.9 * max(write)]
    fk = sum(full_f) / len(full_f)
    wk = sum(full_w) / len(full_w)
    algo = frames * bpf
    res = {
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {kernel} full-batch "
                  "dispatches; FETCH_SIZE x2 (gfx950 wide-stream correction)",
        "width": W, "height": H, "frames": frames, "mode": mode,
        "fetch_kib_raw": fk, "write_kib": wk,
        "read_bytes_per_launch": 2 * fk * 1024, "write_bytes_per_launch": wk * 1024,
        "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
        "algorithmic_bytes_per_launch": algo,
        "traffic_over_algorithmic": (2 * fk * 1024 + wk * 1024) / algo,
        "dispatches": [len(full_f), len(full_w)],
        "kernel": kernel,
        "lib_sha256": lib_sha256(),
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
