#!/bin/bash
# GRAY8 table kernel: 16 vs 12 waves per group with the map (the 16-wave map
# kernels spill) and without, both modes.
set -o pipefail
OUT=gpurun_out/${1:-r03graymap}
mkdir -p $OUT
for cfg in "overall map" "pf map" "overall nomap"; do
  timeout -k 10 300 python -u tools/gray_variant_ab.py 3 6000 4,a0w12 $cfg >> $OUT/gray_waves_ab.jsonl 2>> $OUT/gray_waves_ab.err || exit 1
done
cat $OUT/gray_waves_ab.jsonl
