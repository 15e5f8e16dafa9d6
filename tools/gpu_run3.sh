#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 240 ./build/probe 1000 5 > gpurun_out/probe3.txt 2>&1
rc=$?; cat gpurun_out/probe3.txt; exit $rc
