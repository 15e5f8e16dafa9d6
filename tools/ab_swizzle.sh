#!/bin/bash
# GRAY8 table swizzle A/B: GPU parity of the gray series with the swizzled
# library, then tools/content_rate.py (gray kernel) alternated between
# build/var_noswz (unswizzled table) and build/var_swz over two rounds.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/swz
for v in noswz swz; do [ -f build/var_$v/libdips_hip.so ] || { echo "missing build/var_$v"; exit 1; }; done
cp dips_amd/lib/libdips_hip.so gpurun_out/swz/shipped.so
trap 'cp gpurun_out/swz/shipped.so dips_amd/lib/libdips_hip.so' EXIT
cp build/var_swz/libdips_hip.so dips_amd/lib/libdips_hip.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_series.py -k "gray" > gpurun_out/swz/pytest.txt 2>&1
rc=$?; tail -3 gpurun_out/swz/pytest.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for v in noswz swz; do
  cp build/var_$v/libdips_hip.so dips_amd/lib/libdips_hip.so
  CONTENT_KERNELS=gray timeout -k 10 200 python -u tools/content_rate.py > gpurun_out/swz/${v}_$r.jsonl 2> gpurun_out/swz/${v}_$r.err
  rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/swz/${v}_$r.err; exit $rc; }
  echo "$v r$r: $(python3 -c 'import sys,json;print([(json.loads(l)["content"],json.loads(l)["frac_of_8TBps"]) for l in open(sys.argv[1])])' gpurun_out/swz/${v}_$r.jsonl)"
done; done
