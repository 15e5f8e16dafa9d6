#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_compat.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/cb_pytest.txt 2>&1; rc=$?
tail -5 gpurun_out/cb_pytest.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/cb_pytest.txt; exit $rc; }
timeout -k 10 300 python -u tools/compat_bench.py > gpurun_out/compat_bench.jsonl 2> gpurun_out/compat_bench.err; rc=$?
cat gpurun_out/compat_bench.jsonl; [ $rc -ne 0 ] && { tail -30 gpurun_out/compat_bench.err; exit $rc; }
exit 0
