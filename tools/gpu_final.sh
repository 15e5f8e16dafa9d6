#!/bin/bash
# Round-end GPU evidence: all GPU tests, smoke(), the headline bench with its
# rocprofv3 kernel-trace stats and PMC traffic, and the same for the dips_alt
# batch kernel.  Every step has its own time limit; the first failure ends it.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/final_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/final_pytest_gpu.txt; [ $rc -ne 0 ] && { tail -60 gpurun_out/final_pytest_gpu.txt; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1; rc=$?
cat gpurun_out/final_smoke.txt; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench_full.sh; rc=$?; [ $rc -ne 0 ] && exit $rc
bash profiles/collect_alt_pmc.sh 1000; rc=$?; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/alt_pmc_traffic.json profiles/alt_pmc_traffic.json
timeout -k 10 300 python -u tools/alt_bench.py > gpurun_out/final_alt_bench.json 2> gpurun_out/final_alt_bench.err; rc=$?
cat gpurun_out/final_alt_bench.json; [ $rc -ne 0 ] && { tail -20 gpurun_out/final_alt_bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_alt_final -o alt -- \
  python3 tools/alt_bench.py > gpurun_out/final_alt_bench_rocprof.json 2> gpurun_out/final_alt_bench_rocprof.err; rc=$?
cat gpurun_out/final_alt_bench_rocprof.json; exit $rc
