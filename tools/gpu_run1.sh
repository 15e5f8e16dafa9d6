#!/bin/bash
# First GPU pass: smoke, GPU tests, short bench, rocprof kernel stats.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"
if [ $rc -ge 124 ] || [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --frames-per-gpu 1000 --steps 5 --warmup 2 --cpu-seconds 5 > gpurun_out/bench_short.json 2> gpurun_out/bench_short.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_short.json
exit $rc
