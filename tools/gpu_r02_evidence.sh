#!/bin/bash
# Round-2 GPU evidence, part A: every GPU test, smoke(), the headline bench,
# its rocprofv3 kernel-trace stats and PMC HBM traffic (keyed to this
# library build).  Part B (tools/gpu_r02_evidence_b.sh): sustained 100-step
# run, SQ counters, the config sweep, the visual-operator benches.
# Every GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r02_pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/r02_pytest_gpu.txt; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.txt 2>&1; rc=$?
cat gpurun_out/r02_smoke.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench_full.sh
