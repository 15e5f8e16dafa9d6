set -e
mkdir -p gpurun_out
for r in 1 2; do for v in base d4 w5 w6; do
  cp build/var_$v/libdips_hip.so dips_amd/lib/libdips_hip.so
  timeout -k 10 200 python -u tools/config_sweep.py > gpurun_out/ab_${v}_$r.jsonl 2>gpurun_out/ab_${v}_$r.err
  echo "$v r$r: $(grep -E 'gray8|configs\[2\]' gpurun_out/ab_${v}_$r.jsonl | python3 -c 'import sys,json;print([(json.loads(l)["config"][:20],json.loads(l)["frac_of_8TBps"],json.loads(l)["first_frames_match_oracle"]) for l in sys.stdin])')"
done; done
