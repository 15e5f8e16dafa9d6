#!/bin/bash
# LDS counters of the GRAY8 table kernel (series_gray_lut_kernel, 4K gray8
# 'per-frame', 15000 frames via tools/config_sweep.py), one counter set per
# rocprofv3 pass (--pmc only, <= 8 SQ counters), summarised by
# tools/pmc_kernel_summary.py.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcgray}; rm -rf $OUT; mkdir -p $OUT
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS" \
           "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- \
    python3 tools/config_sweep.py --only "gray8, 15000" --steps 2 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_kernel_summary.py $OUT series_gray_lut_kernel > $OUT/summary.txt; rc=$?; cat $OUT/summary.txt; exit $rc
