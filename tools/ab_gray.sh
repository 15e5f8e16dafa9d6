#!/bin/bash
# A/B of series library builds on the GPU box: build/var_<v>/libdips_hip.so
# for v in base d4 w5 w6, built here beforehand with
#   make -C dips_amd/csrc OBJDIR=../../build/var_<v>/obj OUTDIR=../../build/var_<v> \
#        HIPFLAGS="<default flags> -DDIPS_DEPTH_GRAY=4 | -DDIPS_MIN_WAVES_PER_SIMD=5|6"
# (base = a copy of the shipped library).  Each variant runs the whole config
# sweep, alternated over two rounds; the shipped library is restored at the end.
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in base d4 w5 w6; do [ -f build/var_$v/libdips_hip.so ] || { echo "missing build/var_$v"; exit 1; }; done
cp dips_amd/lib/libdips_hip.so gpurun_out/shipped_libdips_hip.so
trap 'cp gpurun_out/shipped_libdips_hip.so dips_amd/lib/libdips_hip.so' EXIT
for r in 1 2; do for v in base d4 w5 w6; do
  cp build/var_$v/libdips_hip.so dips_amd/lib/libdips_hip.so
  timeout -k 10 200 python -u tools/config_sweep.py > gpurun_out/ab_${v}_$r.jsonl 2>gpurun_out/ab_${v}_$r.err
  echo "$v r$r: $(grep -E 'gray8|configs\[2\]' gpurun_out/ab_${v}_$r.jsonl | python3 -c 'import sys,json;print([(json.loads(l)["config"][:20],json.loads(l)["frac_of_8TBps"],json.loads(l)["first_frames_match_oracle"]) for l in sys.stdin])')"
done; done
