#!/bin/bash
# GPU round for the dips_alt operator: GPU tests (all), the alt bench, a
# rocprofv3 kernel-trace of the alt bench, and a short headline bench.py run
# (regression check of the series kernel after the intensity_v2.h move).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/alt_pytest_gpu.txt 2>&1; rc=$?
tail -5 gpurun_out/alt_pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/alt_pytest_gpu.txt; exit $rc; }
timeout -k 10 300 python -u tools/alt_bench.py > gpurun_out/alt_bench.json 2> gpurun_out/alt_bench.err; rc=$?
cat gpurun_out/alt_bench.json; [ $rc -ne 0 ] && { tail -30 gpurun_out/alt_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_alt -o alt -- \
  python3 tools/alt_bench.py --steps 3 --warmup 1 > gpurun_out/alt_bench_rocprof.json 2> gpurun_out/alt_bench_rocprof.err; rc=$?
cat gpurun_out/alt_bench_rocprof.json; [ $rc -ne 0 ] && { tail -30 gpurun_out/alt_bench_rocprof.err; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err; rc=$?
cat gpurun_out/bench_quick.json; [ $rc -ne 0 ] && { tail -30 gpurun_out/bench_quick.err; exit $rc; }
exit 0
