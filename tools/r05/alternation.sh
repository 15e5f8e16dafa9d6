#!/bin/bash
# Consecutive processes, each with one 124 GB frame buffer
# (tools/r05/alternation_probe.py): six without waiting, then six that wait
# for the device's memory to be free before allocating.  Each process has
# its own time limit; the first failure ends the script.
cd "$(dirname "$0")/../.."
O=gpurun_out/${1:-alternation}
mkdir -p $O
for w in 0 20; do
  for i in 1 2 3 4 5 6; do
    timeout -k 10 120 python -u tools/r05/alternation_probe.py $w >> $O/wait$w.jsonl 2>> $O/wait$w.err || exit $?
    tail -1 $O/wait$w.jsonl
  done
done
exit 0
