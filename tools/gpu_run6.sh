#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for n in salu f64 w5 f64w5 f64same; do
  timeout -k 10 200 ./build/probe_$n 1000 5 "U=4" > gpurun_out/probe_$n.txt 2>&1
  rc=$?; echo "== $n rc=$rc"; cat gpurun_out/probe_$n.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
