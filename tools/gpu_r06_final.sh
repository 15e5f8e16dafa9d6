#!/bin/bash
# Round-6 evidence for the committed library: the given GPU tests, PMC
# traffic of the headline kernel (keyed to this library's sha256), the
# driver's bench command, and the bench under rocprofv3 kernel-trace stats.
# Each GPU step has its own time limit; the first failure ends the script.
# Usage: bash tools/gpu_r06_final.sh OUTDIR [pytest targets...]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-r06final}
shift
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 600 --timeout-method thread \
    > $O/pytest_gpu.txt 2>&1; rc=$?
  tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
fi
bash profiles/collect_pmc.sh 5000 per-frame; rc=$?; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/pmc_traffic.json $O/pmc_traffic.json
cp gpurun_out/pmc_traffic_map.json $O/pmc_traffic_map.json
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
cp gpurun_out/pmc_traffic_map.json profiles/pmc_traffic_map.json
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json | cut -c1-400; [ $rc -ne 0 ] && { tail -5 $O/bench.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --no-map --no-check --no-legs --no-per-frame-call --no-placement-probe \
  > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.log
rc=$?; echo "rocprof bench rc=$rc"; exit $rc
