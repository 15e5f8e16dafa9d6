#!/bin/bash
# Round 3 stage c2: per-frame / series GPU tests after the keyed zero-copy
# output (2 px/thread), the aligned-load RGB8 kernel and the integer SI;
# then the per-frame A/B, the ragged-batch rates and the integer-SI A/B.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_compat.py \
  tests/test_gpu_sequence.py tests/test_gpu_series.py tests/test_gpu_golden.py > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 400 python3 -u tools/compact_out_ab.py 48 3 > $O/compact_out_ab.jsonl 2> $O/compact_out_ab.err; rc=$?
grep summary $O/compact_out_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $O/compact_out_ab.err; exit $rc; }
timeout -k 10 300 python3 -u tools/keys_tune.py 40 2 > $O/keys_tune.jsonl 2> $O/keys_tune.err; rc=$?
grep summary $O/keys_tune.jsonl | head -6; [ $rc -ne 0 ] && { tail -5 $O/keys_tune.err; exit $rc; }
timeout -k 10 120 python3 -u tools/keys_tune.py 16 trace > /dev/null 2> $O/keys_trace.txt; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/keys_trace.txt; exit $rc; }
timeout -k 10 400 python3 -u tools/fallback_rate.py > $O/fallback_rate.jsonl 2> $O/fallback_rate.err; rc=$?
cat $O/fallback_rate.jsonl; [ $rc -ne 0 ] && { tail -5 $O/fallback_rate.err; exit $rc; }
timeout -k 10 400 python3 -u tools/isi_ab.py 5000 20 3 > $O/isi_ab.jsonl 2> $O/isi_ab.err; rc=$?
cat $O/isi_ab.jsonl; [ $rc -ne 0 ] && { tail -3 $O/isi_ab.err; exit $rc; }
timeout -k 10 400 bash tools/pmc_gray.sh ${O#gpurun_out/}/pmcgray; exit $?
