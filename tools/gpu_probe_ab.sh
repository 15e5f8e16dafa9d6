#!/bin/bash
# A/B of two probe builds (build/probe vs build/$1), alternating processes.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
B=${1:-probe_exec}; FILT=${2:-kUnrollV2}
for r in 1 2; do
  for p in probe $B; do
    timeout -k 10 200 ./build/$p 1000 5 "$FILT" > gpurun_out/ab_${p}_$r.txt 2>&1 || { echo "$p rc=$?"; cat gpurun_out/ab_${p}_$r.txt; exit 1; }
    echo "== $p run $r"; grep -v "^  frame" gpurun_out/ab_${p}_$r.txt
  done
done
