#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_alt.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/feed_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/feed_pytest.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/feed_pytest.txt; exit $rc; }
timeout -k 10 300 python -u tools/host_feed_rate.py 160 > gpurun_out/host_feed_rate.jsonl 2> gpurun_out/host_feed_rate.err; rc=$?
cat gpurun_out/host_feed_rate.jsonl; [ $rc -ne 0 ] && { tail -20 gpurun_out/host_feed_rate.err; exit $rc; }
timeout -k 10 300 python -u tools/compat_bench.py > gpurun_out/compat_bench2.jsonl 2> gpurun_out/compat_bench2.err; rc=$?
cat gpurun_out/compat_bench2.jsonl; exit $rc
