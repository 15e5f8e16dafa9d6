#!/bin/bash
# per_frame_call leg with a small and a full resident batch beside it
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03pfc}
mkdir -p $O
for F in 100 5000 100; do
  timeout -k 10 400 python3 bench.py --frames-per-gpu $F --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --no-map \
    --no-legs > $O/pfc_$F.json 2> $O/pfc_$F.log; rc=$?
  [ $rc -ne 0 ] && { tail -5 $O/pfc_$F.log; exit $rc; }
  python3 -c "import json;b=json.load(open('$O/pfc_$F.json'));print($F, b['per_frame_call']['frames_per_s'], b['per_frame_call']['ms_per_call_median'])"
done
DIPS_COPY_THREADS=8 timeout -k 10 120 python3 -u tools/callback_rate_once.py 64
