#!/bin/bash
# SQ counters of the v2 series kernel (real frames and compute-only build).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcv2; mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY" "SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU"; do
  for b in probe probe_same; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/$b.$i -o run -- ./build/$b 1000 2 "v2<U=kUnrollV2,PF=true>" > $OUT/$b.$i.log 2>&1
    rc=$?; echo "$b $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$b.$i.log; exit $rc; }
  done
done
exit 0
