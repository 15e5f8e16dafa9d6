#!/bin/bash
# Round-4 first GPU pass: the RGBA8 cross-lane realignment against the
# oracle (unaligned / offset / fuzz tests), the new parity tests (timed
# configuration at 4K, bench N > 1 rehearsal on the part-major schedule,
# failure path), the alignment rate sweep, the read-walk shape probe, the
# per-frame-call copy-pool A/B, then a bench line.  Each GPU step has its own
# limit; the first failure ends the script.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  tests/test_gpu_fuzz.py tests/test_gpu_compact_io.py -k "unaligned or intensity_sum_forms or fuzz or random or zero_copy" > $O/pytest_align.txt 2>&1; rc=$?
tail -5 $O/pytest_align.txt; [ $rc -ne 0 ] && { tail -80 $O/pytest_align.txt; exit $rc; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_gpu_timed_config.py tests/test_gpu_bench_rehearsal.py > $O/pytest_new.txt 2>&1; rc=$?
tail -15 $O/pytest_new.txt; [ $rc -ne 0 ] && { tail -80 $O/pytest_new.txt; exit $rc; }
timeout -k 10 300 python -u tools/fallback_rate.py > $O/fallback_rate.jsonl 2> $O/fallback_rate.err; rc=$?
cat $O/fallback_rate.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 tools/read_walk_probe 5000 > $O/read_walk_shapes.jsonl 2> $O/read_walk.err; rc=$?
cat $O/read_walk_shapes.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/pfc_threads_ab.py --rounds 2 > $O/pfc_threads_ab.jsonl 2> $O/pfc.err; rc=$?
cat $O/pfc_threads_ab.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json; tail -5 $O/bench.log; exit $rc
