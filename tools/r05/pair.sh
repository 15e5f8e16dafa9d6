#!/bin/bash
# A 1 GiB-aligned virtual-memory frame buffer (v) against torch's default
# one (d), both in one process, measured alternately; three consecutive
# processes with the allocation order swapped (tools/placement_probe.py
# --pair).  Each process has its own time limit; the first failure ends it.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-pair}
mkdir -p $O
for i in 1 2 3 4; do
  ord=vd; [ $((i % 2)) -eq 0 ] && ord=dv
  timeout -k 10 180 python -u tools/placement_probe.py --pair $ord --slices 4 > $O/proc${i}_$ord.jsonl 2> $O/proc${i}_$ord.err
  rc=$?; cut -c1-170 $O/proc${i}_$ord.jsonl; [ $rc -ne 0 ] && { tail -5 $O/proc${i}_$ord.err; exit $rc; }
done
exit 0
