#!/bin/bash
# Round 3: zero-copy per-frame output as keys -- the per-frame GPU tests,
# then the in-process A/B (tools/compact_out_ab.py).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03compact}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compat.py \
  tests/test_gpu_sequence.py > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 400 python3 -u tools/compact_out_ab.py 48 3 > $O/compact_out_ab.jsonl 2> $O/compact_out_ab.err; rc=$?
cat $O/compact_out_ab.jsonl | grep summary; tail -3 $O/compact_out_ab.err; exit $rc
