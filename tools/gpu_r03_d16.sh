#!/bin/bash
# Round 3 (session 2): GRAY8 layout 4 (layout 3 with d16 LDS gathers): the gray
# GPU tests, then the in-process A/B against layout 3 (synthetic clip and
# i.i.d. random frames).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03d16}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py -k gray \
  > $O/pytest_gray.txt 2>&1; rc=$?
tail -3 $O/pytest_gray.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_gray.txt; exit $rc; }
timeout -k 10 400 python -u tools/gray_variant_ab.py 3 6000 L3,L4 pf nomap synth > $O/gray_d16_ab.jsonl 2> $O/gray_d16_ab.err
rc=$?; cat $O/gray_d16_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $O/gray_d16_ab.err; exit $rc; }
timeout -k 10 300 python -u tools/gray_variant_ab.py 2 6000 L3,L4 pf nomap random > $O/gray_d16_ab_random.jsonl 2> $O/gray_d16_ab_random.err
rc=$?; cat $O/gray_d16_ab_random.jsonl; [ $rc -ne 0 ] && { tail -5 $O/gray_d16_ab_random.err; exit $rc; }
exit 0
