#!/bin/bash
cd "$(dirname "$0")/.."
for n in probe_same probe_samenored probe_nored; do
  timeout -k 10 200 ./build/$n 1000 5 "series<U=4,D=2" > gpurun_out/$n.txt 2>&1
  rc=$?; echo "== $n rc=$rc"; cat gpurun_out/$n.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
