#!/bin/bash
# HBM traffic of the series kernel from rocprofv3 PMC counters, one counter
# set per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# --pmc only (no sys/runtime traces).  Writes profiles/pmc_traffic.json,
# which bench.py reports as roofline.traffic.
# Usage (on the GPU box): bash profiles/collect_pmc.sh [frames] [mode]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
F=${1:-5000}
MODE=${2:-per-frame}
OUT=gpurun_out/pmc_bench
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 bench.py --frames-per-gpu $F --steps 2 --warmup 1 --mode $MODE --no-cpu-baseline --no-pcie \
    --no-tau0 --no-legs --no-per-frame-call --no-placement-probe --map-frames 2500 > $OUT/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
PF=$([ "$MODE" = per-frame ] && echo true || echo false)
python3 tools/pmc_to_json.py $OUT $F $MODE gpurun_out/pmc_traffic.json \
  "series_v2_kernel<3, 0, 5, $PF, false, false, 1>" && \
python3 tools/pmc_to_json.py $OUT 2500 $MODE gpurun_out/pmc_traffic_map.json \
  "series_v2_kernel<3, 0, 5, $PF, true, false, 1>" $((3840 * 2160 * 3 * 2))
# copy gpurun_out/pmc_traffic*.json into profiles/ after merge-back
