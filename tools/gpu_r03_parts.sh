#!/bin/bash
# Round 3 (session 2): the part-major schedule of the RGB8 / RGBA8 series
# kernel as the library default.  Every GPU test, then the in-process A/B
# against the contiguous ranges (hipEvent time + SMU energy), per-frame and
# overall, then the default bench line.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03parts}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 400 python -u tools/isi_ab.py 5000 20 4 per-frame parts,contig > $O/parts_ab_pf.jsonl 2> $O/parts_ab_pf.err
rc=$?; cat $O/parts_ab_pf.jsonl; [ $rc -ne 0 ] && { tail -5 $O/parts_ab_pf.err; exit $rc; }
timeout -k 10 300 python -u tools/isi_ab.py 5000 20 2 overall parts,contig > $O/parts_ab_overall.jsonl 2> $O/parts_ab_overall.err
rc=$?; cat $O/parts_ab_overall.jsonl; [ $rc -ne 0 ] && { tail -5 $O/parts_ab_overall.err; exit $rc; }
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-per-frame-call > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json | cut -c1-600; [ $rc -ne 0 ] && { tail -5 $O/bench.log; exit $rc; }
exit 0
