#!/bin/bash
# Round-4 pass n: the layout-4 sample on each item's second frame pair;
# parity, the five GRAY8 contents (2 / 5 / 4), configs[0] by kernel form, and
# the series cleared by the kernel vs a fill launch on the headline (alternated
# in one process).
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04n}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_series.py \
  tests/test_gpu_timed_config.py -k "gray or dirty or part_major or timed_config" > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest.txt; exit $rc; }
LAYOUTS=${LAYOUTS:-2,5,4} timeout -k 10 400 python -u tools/gray_layout_ab.py > $O/gray_layout_ab.jsonl 2> $O/gray.err || exit $?
for g in auto band5 lut16 f32 auto; do
  timeout -k 10 120 python -u tools/config_sweep.py --only "configs[0]" --steps 50 --gray-kernel $g >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
done
timeout -k 10 400 python -u tools/isi_ab.py 5000 10 4 per-frame kzero,fill > $O/kzero_ab.jsonl 2> $O/ab.err; rc=$?
tail -1 $O/kzero_ab.jsonl | cut -c1-300; exit $rc
