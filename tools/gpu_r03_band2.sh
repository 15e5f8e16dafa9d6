#!/bin/bash
# Round 3 (session 2): LDS / SQ counters of the GRAY8 table kernel, layout 3
# against layout 2, then the vecs-per-lane sweep of layout 3 in one process.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03band2}
mkdir -p $O
bash tools/pmc_gray_band.sh ${1:-r03band2}/pmc > $O/pmc.txt 2>&1; rc=$?
cat $O/pmc.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/gray_variant_ab.py 3 6000 L3,L3u3,L3u2 pf nomap synth > $O/gray_band_u.jsonl 2> $O/gray_band_u.err
rc=$?; cat $O/gray_band_u.jsonl; [ $rc -ne 0 ] && { tail -5 $O/gray_band_u.err; exit $rc; }
exit 0
