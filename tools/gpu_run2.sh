#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --frames-per-gpu 2000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_pf.json 2> gpurun_out/bench_pf.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_pf.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --frames-per-gpu 2000 --steps 5 --warmup 2 --no-cpu-baseline --mode overall > gpurun_out/bench_ov.json 2> gpurun_out/bench_ov.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_ov.json; exit $rc
