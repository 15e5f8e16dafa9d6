#!/bin/bash
# SQ / LDS counters of the GRAY8 table kernel, layout 3 (band clamp, the
# default) and layout 2 ((a, b) table), 4K gray8 per-frame, 15000 frames via
# tools/config_sweep.py.  One counter set per rocprofv3 pass (--pmc only),
# summarised by tools/pmc_kernel_summary.py.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcgrayband}; rm -rf $OUT; mkdir -p $OUT
for v in "3 16" "2 16"; do
  set -- $v
  export DIPS_GRAY_LUT=$1 DIPS_GRAY_ALU=0
  D=$OUT/L$1; mkdir -p $D
  i=0
  for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
             "GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $D/p$i -o run -- \
      python3 tools/config_sweep.py --only "gray8, 15000" --steps 2 > $D/p$i.log 2>&1
    rc=$?; echo "L$1 pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $D/p$i.log; exit $rc; }
  done
  python3 tools/pmc_kernel_summary.py $D series_gray_lut_kernel > $D/summary.json || exit 1
  python3 - $D/summary.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); c=d["counters"]; g=c.get("GRBM_GUI_ACTIVE",0)/8
out={"dur_ms":round(d["duration_s_profiled"]*1e3,3)}
for k in ("SQ_INSTS_LDS","SQ_INSTS_VALU","SQ_INSTS_SALU"):
    out[k]=c.get(k)
if g:
    out["clk_GHz"]=round(g/d["duration_s_profiled"]/1e9,3)
    for k in ("SQ_LDS_IDX_ACTIVE","SQ_ACTIVE_INST_LDS","SQ_BUSY_CYCLES"):
        if k in c: out[k+"_per_cu_frac"]=round(c[k]/256/g,3)
    for k in ("SQ_WAVE_CYCLES","SQ_WAIT_INST_LDS","SQ_WAIT_INST_ANY","SQ_ACTIVE_INST_ANY","SQ_ACTIVE_INST_VALU"):
        if k in c and c.get("SQ_WAVES"): out[k+"_per_wave_frac"]=round(c[k]/c["SQ_WAVES"]/g,3)
if c.get("SQ_INSTS_LDS"): out["conflict_per_lds"]=round(c.get("SQ_LDS_BANK_CONFLICT",0)/c["SQ_INSTS_LDS"],3)
print(json.dumps(out))
PY
done
