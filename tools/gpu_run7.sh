#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
for n in probe probe_same; do
  timeout -k 10 200 ./build/$n 1000 5 "U=4" > gpurun_out/$n.txt 2>&1
  rc=$?; echo "== $n rc=$rc"; cat gpurun_out/$n.txt; [ $rc -ne 0 ] && exit $rc
done
exit 0
