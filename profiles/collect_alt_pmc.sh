#!/bin/bash
# HBM traffic of the dips_alt batch kernel (tools/alt_bench.py workload) from
# rocprofv3 PMC counters, one counter per pass, --pmc only.  Writes
# gpurun_out/alt_pmc_traffic.json (copy into profiles/ after merge-back).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
F=${1:-1000}
OUT=gpurun_out/pmc_alt
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python3 tools/alt_bench.py --frames $F --steps 2 --warmup 1 > $OUT/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_to_json.py $OUT $F run-loop gpurun_out/alt_pmc_traffic.json alt_batch_kernel $((3840*2160*8))
