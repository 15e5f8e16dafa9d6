import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l)
    g=d.get("gpu") or {}
    print(d.get("class",d.get("phase")), d.get("pJ_per_wave64_instr_above_idle"), g.get("avg_power_W_energy"), g.get("gfxclk_MHz_mean"), g.get("ppt_residency_frac"), "%.3g" % d.get("wave_instr_per_s",0))
