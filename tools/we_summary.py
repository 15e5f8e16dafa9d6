import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    g = d.get("gpu") or {}
    print(d["round"], "%-7s" % d["schedule"], d["frac_of_8TBps"], d.get("mJ_per_frame"), g.get("avg_power_W_energy"),
          g.get("gfxclk_MHz_mean"), g.get("ppt_residency_frac"))
