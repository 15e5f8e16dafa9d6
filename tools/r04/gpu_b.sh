#!/bin/bash
# Round-4 second GPU pass: the whole GPU suite (RGBA8 realignment and GRAY8
# auto layout now library defaults), the per-frame-call path A/B (zero-copy
# vs copy engines, pool threads), the GRAY8 layout A/B over contents.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 560 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -80 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 380 python -u tools/pfc_threads_ab.py --rounds 2 --variants 8:0:1:0,8:0:2:0,12:0:2:0,8:0:1:1,8:0:2:1,16:0:2:1 \
  > $O/pfc_path_ab.jsonl 2> $O/pfc.err; rc=$?
cat $O/pfc_path_ab.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 220 python -u tools/gray_layout_ab.py > $O/gray_layout_ab.jsonl 2> $O/gray.err; rc=$?
cat $O/gray_layout_ab.jsonl; exit $rc
