#!/bin/bash
# Round 3 (session 2): the GRAY8 band-clamp table (layout 3) and the batched
# reduce.  Every GPU test, then the in-process layout A/B on the bench's
# synthetic clip and on i.i.d. random frames, then the default bench line.
# Each GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03band}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 400 python -u tools/gray_variant_ab.py 3 6000 L3,L2 pf nomap synth > $O/gray_band_ab.jsonl 2> $O/gray_band_ab.err
rc=$?; cat $O/gray_band_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $O/gray_band_ab.err; exit $rc; }
timeout -k 10 300 python -u tools/gray_variant_ab.py 2 6000 L3,L2 pf nomap random > $O/gray_band_ab_random.jsonl 2> $O/gray_band_ab_random.err
rc=$?; cat $O/gray_band_ab_random.jsonl; [ $rc -ne 0 ] && { tail -5 $O/gray_band_ab_random.err; exit $rc; }
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-per-frame-call > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.log; exit $rc; }
exit 0
