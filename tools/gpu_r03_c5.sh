#!/bin/bash
# Round 3 stage c5: GPU timeline of the per-frame call's stripe kernels.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c5}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- \
  python3 tools/keys_tune.py 16 trace > $O/trace_stdout.txt 2> $O/keys_trace.txt; rc=$?
[ $rc -ne 0 ] && { tail -5 $O/keys_trace.txt; exit $rc; }
python3 tools/kernel_timeline.py $O/kt compat_main_host 150 > $O/timeline.txt; cat $O/timeline.txt; tail -4 $O/keys_trace.txt
