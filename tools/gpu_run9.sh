#!/bin/bash
cd "$(dirname "$0")/.."
for n in abl_base abl_nothr abl_vcnt abl_f32 abl_nou abl_nored; do
  timeout -k 10 200 ./build/probe_$n 1000 5 "series<U=4,D=2" > gpurun_out/probe_$n.txt 2>&1
  rc=$?; echo "== $n rc=$rc"; cat gpurun_out/probe_$n.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
