#!/bin/bash
# Every BASELINE.json config under rocprofv3: kernel trace + stats, then the
# FETCH_SIZE and WRITE_SIZE passes (one counter set per pass, --pmc only),
# each a run of tools/config_sweep.py with its own time limit.  Summarised by
# tools/r05/sweep_summary.py.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${1:-sweep_prof}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 tools/config_sweep.py --steps 3 --no-placement-probe > $O/kt.jsonl 2> $O/kt.err || { echo "kt rc=$?"; tail -5 $O/kt.err; exit 1; }
echo "kernel trace ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --output-format csv -d $O/$c -o run -- \
    python3 tools/config_sweep.py --steps 2 --no-placement-probe > $O/$c.jsonl 2> $O/$c.err || { echo "$c rc=$?"; tail -5 $O/$c.err; exit 1; }
  echo "$c ok"
done
python3 tools/r05/sweep_summary.py $O > $O/summary.txt && cat $O/summary.txt
