#!/bin/bash
# Effective clock of kernel variants: GRBM_GUI_ACTIVE / 8 XCDs / duration.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/clk; mkdir -p $OUT
for n in probe probe_same; do
  timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/$n -o run -- ./build/$n 1000 3 "U=4,D=2,PF=true" > $OUT/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/walk -o run -- ./build/probe 1000 3 "walk" > $OUT/walk.log 2>&1
echo "walk rc=$?"
