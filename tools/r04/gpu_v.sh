#!/bin/bash
# Round-4 pass v: merged partial records (DIPS_SERIES_MERGE=1): parity, then
# merged vs unmerged alternated in one process at 4K per-frame and overall.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04v}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  -k "merged" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest.txt; exit $rc; }
timeout -k 10 500 python -u tools/isi_ab.py 5000 10 4 per-frame merge,nomerge > $O/merge_ab_pf.jsonl 2> $O/ab.err || exit $?
tail -1 $O/merge_ab_pf.jsonl | cut -c1-500
timeout -k 10 500 python -u tools/isi_ab.py 5000 10 4 overall merge,nomerge > $O/merge_ab_ov.jsonl 2>> $O/ab.err || exit $?
tail -1 $O/merge_ab_ov.jsonl | cut -c1-500
