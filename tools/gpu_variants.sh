#!/bin/bash
# GPU check of the visual table kernels' (U, D) variants: the compat and alt
# GPU tests on the shipped defaults, then the in-process variant A/Bs.
cd "$(dirname "$0")/.."
O=gpurun_out/var; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_compat.py tests/test_gpu_alt.py > $O/pytest.txt 2>&1
rc=$?; tail -2 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/compat_variant_ab.py 3 22,33,43,44 > $O/compat_ab.jsonl 2> $O/compat_ab.err
rc=$?; cut -c1-150 $O/compat_ab.jsonl; [ $rc -ne 0 ] && { tail -3 $O/compat_ab.err; exit $rc; }
timeout -k 10 240 python -u tools/alt_variant_ab.py 3 22,23,33,42,43 > $O/alt_ab.jsonl 2> $O/alt_ab.err
rc=$?; cut -c1-150 $O/alt_ab.jsonl; [ $rc -ne 0 ] && tail -3 $O/alt_ab.err; exit $rc
