#!/bin/bash
# Round-4 pass l: the part-major schedule for 'overall' batches
# (DIPS_SERIES_PARTS=2): parity, then an in-process A/B at 4K overall.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_series.py \
  -k "part_major" > $O/pytest_parts.txt 2>&1; rc=$?
tail -3 $O/pytest_parts.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_parts.txt; exit $rc; }
timeout -k 10 400 python -u tools/isi_ab.py 5000 10 3 overall contig,partsall > $O/overall_parts_ab.jsonl 2> $O/ab.err; rc=$?
cat $O/overall_parts_ab.jsonl; exit $rc
