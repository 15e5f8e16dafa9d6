#!/bin/bash
# Round-2 GPU evidence, part B (see tools/gpu_r02_evidence.sh).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-pcie --no-map \
  > gpurun_out/r02_sustain_steps100.json 2> gpurun_out/r02_sustain_steps100.log; rc=$?
cat gpurun_out/r02_sustain_steps100.json; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_sq.sh; rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/config_sweep.py > gpurun_out/r02_config_sweep.jsonl 2> gpurun_out/r02_config_sweep.err; rc=$?
cat gpurun_out/r02_config_sweep.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/alt_bench.py > gpurun_out/r02_alt_bench.json 2> gpurun_out/r02_alt_bench.err; rc=$?
cat gpurun_out/r02_alt_bench.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/compat_bench.py --kernels lut > gpurun_out/r02_compat_bench.jsonl 2> gpurun_out/r02_compat_bench.err; rc=$?
cat gpurun_out/r02_compat_bench.jsonl; exit $rc
