#!/bin/bash
# dips_alt fast epilogue: exhaustive device check, alt GPU tests, alt bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 ./build/altcheck > gpurun_out/altcheck.txt 2>&1; rc=$?
cat gpurun_out/altcheck.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_alt.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/alt2_pytest.txt 2>&1; rc=$?
tail -5 gpurun_out/alt2_pytest.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/alt2_pytest.txt; exit $rc; }
timeout -k 10 300 python -u tools/alt_bench.py > gpurun_out/alt2_bench.json 2> gpurun_out/alt2_bench.err; rc=$?
cat gpurun_out/alt2_bench.json; [ $rc -ne 0 ] && { tail -30 gpurun_out/alt2_bench.err; exit $rc; }
exit 0
