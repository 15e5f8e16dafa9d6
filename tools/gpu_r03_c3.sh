#!/bin/bash
# Round 3 stage c3: per-frame call tuning -- huge-page pinned buffers A/B,
# stripe geometry with one pixel per thread, traces of both buffer kinds.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compat.py \
  tests/test_gpu_sequence.py > $O/pytest_gpu.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.txt; exit $rc; }
DIPS_PIN_HUGE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_compat.py -k "striped or direct or deferred or resume" > $O/pytest_gpu_huge.txt 2>&1; rc=$?
tail -2 $O/pytest_gpu_huge.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_gpu_huge.txt; exit $rc; }
timeout -k 10 300 python3 -u tools/pin_huge_ab.py 40 4 > $O/pin_huge_ab.jsonl 2> $O/pin_huge_ab.err; rc=$?
cat $O/pin_huge_ab.jsonl | grep summary; [ $rc -ne 0 ] && { tail -5 $O/pin_huge_ab.err; exit $rc; }
timeout -k 10 300 python3 -u tools/keys_tune.py 40 2 > $O/keys_tune.jsonl 2> $O/keys_tune.err; rc=$?
grep summary $O/keys_tune.jsonl | head -8; [ $rc -ne 0 ] && { tail -5 $O/keys_tune.err; exit $rc; }
timeout -k 10 120 python3 -u tools/keys_tune.py 16 trace > /dev/null 2> $O/keys_trace.txt; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/keys_trace.txt; exit $rc; }
DIPS_PIN_HUGE=1 timeout -k 10 120 python3 -u tools/keys_tune.py 16 trace > /dev/null 2> $O/keys_trace_huge.txt; rc=$?
tail -4 $O/keys_trace.txt; tail -4 $O/keys_trace_huge.txt; exit $rc
