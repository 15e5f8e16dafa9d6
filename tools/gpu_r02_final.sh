#!/bin/bash
# Round-2 final GPU evidence for the committed tree: every GPU test, smoke(),
# the headline bench with rocprofv3 kernel-trace stats and PMC traffic, the
# sustained 100-step run, the config sweep, and rocprof stats + PMC traffic
# of the GRAY8 / ComputeState / dips_alt table kernels.  Each GPU step has
# its own time limit; the first failure ends the script.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/final
mkdir -p $O
STAGE=${1:-a}   # a: tests, PMC, headline bench (+ rocprof); b: the rest
if [ "$STAGE" = a ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest_gpu.txt; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?
cat $O/smoke.txt; [ $rc -ne 0 ] && exit $rc
# PMC traffic first, so the bench lines below carry it (keyed to this build)
bash profiles/collect_pmc.sh 5000 per-frame; rc=$?; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/pmc_traffic.json profiles/pmc_traffic.json
cp gpurun_out/pmc_traffic_map.json profiles/pmc_traffic_map.json
bash profiles/collect_alt_pmc.sh 1000; rc=$?; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/alt_pmc_traffic.json profiles/alt_pmc_traffic.json
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.log; rc=$?
cat $O/bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py --no-cpu-baseline --no-pcie --no-map > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.log
rc=$?; echo "rocprof bench rc=$rc"; exit $rc
fi
timeout -k 10 600 python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-pcie --no-map \
  > $O/sustain_steps100.json 2> $O/sustain_steps100.log; rc=$?
cat $O/sustain_steps100.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/config_sweep.py > $O/config_sweep.jsonl 2> $O/config_sweep.err; rc=$?
cat $O/config_sweep.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_gray -o run -- \
  python3 tools/config_sweep.py --only "gray8, 15000" > $O/gray_under_rocprof.jsonl 2> $O/gray_under_rocprof.err
rc=$?; echo "rocprof gray rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/alt_bench.py > $O/alt_bench.json 2> $O/alt_bench.err; rc=$?
cat $O/alt_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_alt -o run -- \
  python3 tools/alt_bench.py > $O/alt_under_rocprof.json 2> $O/alt_under_rocprof.err
rc=$?; echo "rocprof alt rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/compat_bench.py --kernels lut > $O/compat_bench.jsonl 2> $O/compat_bench.err; rc=$?
cat $O/compat_bench.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_compat -o run -- \
  python3 tools/compat_bench.py --kernels lut > $O/compat_under_rocprof.jsonl 2> $O/compat_under_rocprof.err
rc=$?; echo "rocprof compat rc=$rc"; exit $rc
