#!/bin/bash
# Round-5 evidence for the committed library.  Stage a: every GPU test,
# smoke(), PMC traffic of the headline kernel (keyed to this library's
# sha256), the default bench line, the bench under rocprofv3 kernel-trace
# stats.  Stage b: the sustained 100-step bench and the config sweep.  Each
# GPU step has its own time limit; the first failure ends the script.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
STAGE=${1:-a}
O=gpurun_out/${2:-r05final}
mkdir -p $O
if [ "$STAGE" = a ]; then
timeout -k 10 560 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?
cat $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
bash profiles/collect_pmc.sh 5000 per-frame; rc=$?; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
cp gpurun_out/pmc_traffic_map.json profiles/pmc_traffic_map.json
cp gpurun_out/pmc_traffic.json $O/pmc_traffic.json
cp gpurun_out/pmc_traffic_map.json $O/pmc_traffic_map.json
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json; [ $rc -ne 0 ] && { tail -5 $O/bench.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --no-map --no-check --no-legs --no-per-frame-call --no-placement-probe \
  > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.log
rc=$?; echo "rocprof bench rc=$rc"; exit $rc
fi
timeout -k 10 400 python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-pcie --no-map --no-per-frame-call \
  > $O/sustain_steps100.json 2> $O/sustain_steps100.log; rc=$?
cat $O/sustain_steps100.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/config_sweep.py > $O/config_sweep.jsonl 2> $O/config_sweep.err; rc=$?
cat $O/config_sweep.jsonl | cut -c1-200; exit $rc
