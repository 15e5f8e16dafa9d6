#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
grep -oE '^\s*(SQ|TCC|TCP|TA|GRBM)[A-Z0-9_]*' gpurun_out/pmc/counters.txt | sort -u | head -400 > gpurun_out/pmc/counter_names.txt || true
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE SQ_INSTS_VALU_CVT"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/$tag -o run -- ./build/probe 400 2 "$1" > gpurun_out/pmc/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
