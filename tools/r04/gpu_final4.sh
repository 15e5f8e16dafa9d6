#!/bin/bash
# Final evidence for the committed library (stage a of gpu_final.sh), then
# the 'overall' part-major A/B (isi_ab) if time allows.
cd "$(dirname "$0")/../.."
bash tools/r04/gpu_final.sh a r04final4 || exit $?
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 300 python -u tools/isi_ab.py 5000 10 3 overall contig,partsall > $O/overall_parts_ab.jsonl 2> $O/ab.err; rc=$?
tail -1 $O/overall_parts_ab.jsonl; exit $rc
