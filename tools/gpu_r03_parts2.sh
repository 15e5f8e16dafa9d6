#!/bin/bash
# Round 3 (session 2): the part-major schedule in the GRAY8 table kernel too.
# Every GPU test, then the in-process A/B against the contiguous ranges.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03parts2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 400 python -u tools/gray_variant_ab.py 3 6000 L3,L3c pf nomap synth > $O/gray_parts_ab.jsonl 2> $O/gray_parts_ab.err
rc=$?; cat $O/gray_parts_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $O/gray_parts_ab.err; exit $rc; }
exit 0
