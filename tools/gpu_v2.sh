#!/bin/bash
# v2 kernel check on the GPU box: exhaustive intensity check, probe (timing +
# parity vs the previous kernel), compute-only probe, then the GPU tests.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 60 ./build/i2check > gpurun_out/v2_i2check.txt 2>&1; rc=$?
cat gpurun_out/v2_i2check.txt; [ $rc -ne 0 ] && { echo "i2check rc=$rc"; exit $rc; }
timeout -k 10 240 ./build/probe 1000 5 > gpurun_out/v2_probe.txt 2>&1; rc=$?
cat gpurun_out/v2_probe.txt; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
timeout -k 10 240 ./build/probe_same 1000 5 "v2<" > gpurun_out/v2_probe_same.txt 2>&1; rc=$?
cat gpurun_out/v2_probe_same.txt; [ $rc -ne 0 ] && { echo "probe_same rc=$rc"; exit $rc; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/v2_pytest.txt 2>&1; rc=$?
tail -15 gpurun_out/v2_pytest.txt; exit $rc
