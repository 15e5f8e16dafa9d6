#!/bin/bash
# configs[0] (640x480 gray8, 300 frames, tau 0): where the 40 us of a small
# batch go.  Every GRAY8 kernel form through config_sweep, then the default
# under rocprofv3 --kernel-trace --stats (per-kernel durations).
cd "$(dirname "$0")/../.."
O=gpurun_out/r04small; mkdir -p $O
for g in auto band5 lut16 f32 auto; do
  timeout -k 10 120 python -u tools/config_sweep.py --only "configs[0]" --steps 50 --gray-kernel $g >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
done
timeout -k 10 120 python -u tools/config_sweep.py --only "configs[1]" --steps 10 >> $O/sweep.jsonl 2>> $O/sweep.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt -o run -- python3 $GRAFT_REPO_ROOT/tools/config_sweep.py --only "configs[0]" --steps 50 > $GRAFT_REPO_ROOT/$O/kt.log 2>&1
