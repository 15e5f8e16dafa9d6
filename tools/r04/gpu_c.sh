#!/bin/bash
# Round-4 pass c: GRAY8 auto layout with the two-feature choice (band
# fraction, wave spread): its parity tests, then the layout A/B over contents.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  tests/test_gpu_golden.py tests/test_gpu_fuzz.py -k "gray or Gray or golden or random_series or config0 or forms" \
  > $O/pytest_gray.txt 2>&1; rc=$?
tail -3 $O/pytest_gray.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gray.txt; exit $rc; }
timeout -k 10 300 python -u tools/gray_layout_ab.py > $O/gray_layout_ab.jsonl 2> $O/gray.err; rc=$?
cat $O/gray_layout_ab.jsonl; exit $rc
