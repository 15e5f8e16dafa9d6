#!/bin/bash
# Round 3 (session 2): the SADI intensity-sum form of the RGB8 series kernel
# (DIPS_SERIES_ISI=2).  Its parity tests and the series tests, then the
# in-process A/B against the shipped ISI form (hipEvent time + SMU energy),
# per-frame and overall.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03sadi}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  > $O/pytest_series.txt 2>&1; rc=$?
tail -3 $O/pytest_series.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_series.txt; exit $rc; }
timeout -k 10 400 python -u tools/isi_ab.py 5000 20 4 per-frame isi,sadi > $O/sadi_ab_pf.jsonl 2> $O/sadi_ab_pf.err
rc=$?; cat $O/sadi_ab_pf.jsonl; [ $rc -ne 0 ] && { tail -5 $O/sadi_ab_pf.err; exit $rc; }
timeout -k 10 300 python -u tools/isi_ab.py 5000 20 2 overall isi,sadi > $O/sadi_ab_overall.jsonl 2> $O/sadi_ab_overall.err
rc=$?; cat $O/sadi_ab_overall.jsonl; [ $rc -ne 0 ] && { tail -5 $O/sadi_ab_overall.err; exit $rc; }
exit 0
