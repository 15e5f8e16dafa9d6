#!/bin/bash
# SQ / GRBM counters of the headline kernel (series_v2_kernel<3,0,4,PF>, 1000
# 4K RGB8 frames via build/probe) with real frames and the compute-only build
# (build/probe_same: every wave re-reads one frame), one counter set per
# rocprofv3 pass (--pmc only); summarised by tools/sq_summary.py.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcsq; rm -rf $OUT; mkdir -p $OUT
i=0
for set in "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  for b in probe probe_same; do
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/$b.$i -o run -- \
      ./build/$b 1000 2 "U=kUnrollV2,PF=true> tau=8" > $OUT/$b.$i.log 2>&1
    rc=$?; echo "$b pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$b.$i.log; exit $rc; }
  done
done
python3 tools/sq_summary.py $OUT > gpurun_out/sq_summary.txt; rc=$?; cat gpurun_out/sq_summary.txt; exit $rc
