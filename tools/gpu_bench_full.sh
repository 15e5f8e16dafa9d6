#!/bin/bash
# Full bench (defaults) + rocprofv3 kernel-trace stats of the same command + PMC traffic.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 900 python3 bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_full.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --no-map > gpurun_out/prof/bench_kt.json 2> gpurun_out/prof/bench_kt.log
rc=$?; echo "rocprof kt rc=$rc"; cat gpurun_out/prof/bench_kt.json; [ $rc -ne 0 ] && exit $rc
bash profiles/collect_pmc.sh 5000 per-frame
