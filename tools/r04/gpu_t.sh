#!/bin/bash
# Round-4 pass t: HBM traffic (rocprofv3 PMC, one counter per pass, --pmc
# only) of the 4K GRAY8 table kernel (15,000 frames, per-frame) and the 4K
# RGBA8 kernel (3,750 frames, per-frame), through tools/config_sweep.py.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r04t}
mkdir -p $O
for cfg in gray8 RGBA8; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $O/$cfg/$c -o run -- \
      python3 tools/config_sweep.py --only "extra: 3840x2160 $cfg" --steps 2 > $O/${cfg}_$c.log 2>&1
    rc=$?; echo "pmc $cfg $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python3 tools/pmc_to_json.py $O/gray8 15000 per-frame $O/pmc_traffic_gray8.json \
  "series_gray_lut_kernel<4, true, false, 4" $((3840 * 2160)) && \
python3 tools/pmc_to_json.py $O/RGBA8 3750 per-frame $O/pmc_traffic_rgba8.json \
  "series_v2_kernel<4, 0, 4, true, false, false" $((3840 * 2160 * 4)) && \
cat $O/pmc_traffic_gray8.json $O/pmc_traffic_rgba8.json
