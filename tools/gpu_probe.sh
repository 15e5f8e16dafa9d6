#!/bin/bash
# probe only (timing + parity), real frames then the compute-only build.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 240 ./build/probe 1000 5 > gpurun_out/probe.txt 2>&1; rc=$?
cat gpurun_out/probe.txt; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
timeout -k 10 240 ./build/probe_same 1000 5 "v2<" > gpurun_out/probe_same.txt 2>&1; rc=$?
grep -v parity gpurun_out/probe_same.txt | grep -v "^  frame"; exit $rc
