#!/bin/bash
# GPU tests, then the full bench + rocprofv3 kernel stats + PMC traffic.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -30 gpurun_out/pytest_gpu.txt; exit $rc; }
bash tools/gpu_bench_full.sh
