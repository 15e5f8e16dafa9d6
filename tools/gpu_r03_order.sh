#!/bin/bash
# Round 3 (session 2): the interleaved copy-pool order of the zero-copy
# per-frame calls.  The per-frame / ComputeState / dips_alt GPU tests, then
# the in-process order A/B.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03order}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compat.py \
  tests/test_gpu_alt.py tests/test_gpu_sequence.py > $O/pytest_callbacks.txt 2>&1; rc=$?
tail -3 $O/pytest_callbacks.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_callbacks.txt; exit $rc; }
timeout -k 10 400 python -u tools/pfc_order_ab.py 4 208 > $O/pfc_order_ab.jsonl 2> $O/pfc_order_ab.err
rc=$?; cat $O/pfc_order_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $O/pfc_order_ab.err; exit $rc; }
exit 0
