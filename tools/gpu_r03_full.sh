#!/bin/bash
# Round 3: every GPU test, smoke(), then the default bench line.  Each GPU
# step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?
cat $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json; tail -8 $O/bench.log; exit $rc
