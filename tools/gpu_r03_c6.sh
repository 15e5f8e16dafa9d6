#!/bin/bash
# Round 3 stage c6: copy-pool size of the per-frame call (separate processes).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c6}
mkdir -p $O
: > $O/copy_threads.jsonl
for r in 1 2; do
  for n in 8 12 16 6; do
    DIPS_COPY_THREADS=$n timeout -k 10 120 python3 -u tools/callback_rate_once.py 64 >> $O/copy_threads.jsonl 2>> $O/err.txt
    rc=$?; [ $rc -ne 0 ] && { tail -5 $O/err.txt; exit $rc; }
  done
done
cat $O/copy_threads.jsonl; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; exit 0
