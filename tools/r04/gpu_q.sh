#!/bin/bash
# Round-4 pass q: streaming vs plain stores per direction of the per-frame
# call (DIPS_NT_PACK: the packed staging the GPU reads over PCIe right after;
# DIPS_NT_EXPAND: the keys expanded into the caller's output), alternated.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_compact_io.py \
  > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -ne 0 ] && { tail -60 $O/pytest.txt; exit $rc; }
timeout -k 10 900 python -u tools/pfc_threads_ab.py --rounds 4 --calls 300 \
  --env-variants "DIPS_NT_PACK=1,DIPS_NT_EXPAND=1|DIPS_NT_PACK=0,DIPS_NT_EXPAND=1|DIPS_NT_PACK=1,DIPS_NT_EXPAND=0|DIPS_NT_PACK=0,DIPS_NT_EXPAND=0" \
  > $O/nt_dir_ab.jsonl 2> $O/ab.err; rc=$?
python3 - $O/nt_dir_ab.jsonl <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l)
    if "frames_per_s" in r:
        d[json.dumps(r["env"], sort_keys=True)].append((r["frames_per_s"], r["median_ms"], r["p90_ms"], r["phases_ms_median"]["pack_cpu_us"], r["phases_ms_median"]["expand_cpu_us"]))
for k, v in d.items():
    print(k, v)
PY
exit $rc
