#!/bin/bash
# Round 3: the new self-check / legs / per-frame-call bench on one GPU, after
# the GPU tests they rest on.  Each GPU step has its own time limit; the first
# failure ends the script.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard.py \
  "tests/test_gpu_compat.py::test_resume_after_deferred_add_texture" > $O/pytest_gpu.txt 2>&1; rc=$?
tail -15 $O/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json; tail -20 $O/bench.log; exit $rc
