#!/bin/bash
# Interleaved runs of several probe builds (build/<name>...), $ROUNDS rounds,
# variants filtered by $FILT (default: the headline v2 kernel).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FILT=${FILT:-"U=kUnrollV2,PF=true> tau=8"}
for r in $(seq 1 ${ROUNDS:-3}); do
  for p in "$@"; do
    timeout -k 10 200 ./build/$p 1000 5 "$FILT" > gpurun_out/multi_${p}_$r.txt 2>&1 || { echo "$p rc=$?"; cat gpurun_out/multi_${p}_$r.txt; exit 1; }
    echo "== $p run $r: $(grep -E 'median' gpurun_out/multi_${p}_$r.txt)"
  done
done
exit 0
