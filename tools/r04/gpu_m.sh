#!/bin/bash
# Round-4 pass m: layout 4 sampled per workgroup inside the table kernel
# (no probe launch), the series zeroed by the kernels (no fill launch), the
# reduce grid sized to the batch.  Parity first, then the small batch
# (configs[0]) by kernel form, the five GRAY8 contents (2 / 5 / 4), a bench.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  tests/test_gpu_timed_config.py -k "gray or dirty or part_major or timed_config" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest.txt; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
for g in auto band5 lut16 f32 auto; do
  timeout -k 10 120 python -u tools/config_sweep.py --only "configs[0]" --steps 50 --gray-kernel $g >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
done
timeout -k 10 300 python -u tools/config_sweep.py --steps 5 >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
LAYOUTS=${LAYOUTS:-2,5,4} timeout -k 10 400 python -u tools/gray_layout_ab.py > $O/gray_layout_ab.jsonl 2> $O/gray.err || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.log; rc=$?
cut -c1-400 $O/bench.json; exit $rc
