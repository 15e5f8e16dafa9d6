#!/bin/bash
# GRAY8 arithmetic-vec variants: parity tests, then the in-process A/B.
set -o pipefail
OUT=gpurun_out/${1:-r03gray}
VARIANTS=${2:-4,a0w12,a1w12,a2w12}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_gpu_series.py -k "gray" > $OUT/pytest_gray.txt 2>&1 || { tail -30 $OUT/pytest_gray.txt; exit 1; }
tail -3 $OUT/pytest_gray.txt
timeout -k 10 400 python -u tools/gray_variant_ab.py 3 6000 $VARIANTS > $OUT/gray_alu_ab.jsonl 2> $OUT/gray_alu_ab.err
rc=$?; cat $OUT/gray_alu_ab.jsonl; exit $rc
