#!/bin/bash
# Round-4 pass d: GRAY8 layout 5 (band-keyed table without the bank
# swizzle) against 2 / 3 / 4 over the five contents, after its parity tests.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04d}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  -k "gray" > $O/pytest_gray.txt 2>&1; rc=$?
tail -3 $O/pytest_gray.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gray.txt; exit $rc; }
LAYOUTS=${LAYOUTS:-2,3,5,4} timeout -k 10 400 python -u tools/gray_layout_ab.py > $O/gray_layout_ab.jsonl 2> $O/gray.err; rc=$?
cat $O/gray_layout_ab.jsonl | cut -c1-150; exit $rc
