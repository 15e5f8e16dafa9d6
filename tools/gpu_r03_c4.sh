#!/bin/bash
# Round 3 stage c4: packed zero-copy input -- the per-frame GPU tests, the
# in/out A/B, the stripe-geometry sweep and a trace.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c4}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compat.py \
  tests/test_gpu_sequence.py > $O/pytest_gpu.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 400 python3 -u tools/compact_out_ab.py 48 3 > $O/compact_ab.jsonl 2> $O/compact_ab.err; rc=$?
grep summary $O/compact_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $O/compact_ab.err; exit $rc; }
timeout -k 10 300 python3 -u tools/keys_tune.py 40 2 > $O/keys_tune.jsonl 2> $O/keys_tune.err; rc=$?
grep summary $O/keys_tune.jsonl | head -8; [ $rc -ne 0 ] && { tail -5 $O/keys_tune.err; exit $rc; }
timeout -k 10 120 python3 -u tools/keys_tune.py 16 trace > /dev/null 2> $O/keys_trace.txt; rc=$?
tail -4 $O/keys_trace.txt; exit $rc
