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
    > $OUT/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_to_json.py $OUT $F $MODE gpurun_out/pmc_traffic.json  # copy into profiles/ after merge-back
