#!/bin/bash
# A/B of two probe builds (build/probe_old vs build/probe), alternating
# processes, variants filtered by $2 (default: the headline v2 kernel).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
A=${1:-probe_old}; FILT=${2:-"U=kUnrollV2,PF=true> tau=8"}
for r in 1 2 3; do
  for p in $A probe; do
    timeout -k 10 200 ./build/$p 1000 5 "$FILT" > gpurun_out/ab_${p}_$r.txt 2>&1 || { echo "$p rc=$?"; cat gpurun_out/ab_${p}_$r.txt; exit 1; }
    echo "== $p run $r: $(grep -E 'median' gpurun_out/ab_${p}_$r.txt)"
  done
done
exit 0
