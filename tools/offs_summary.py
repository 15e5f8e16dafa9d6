import sys
for l in open(sys.argv[1]):
    p = l.rstrip("\n").split("\t")
    if p[0] == "run":
        ms = float(p[6])
        print(sys.argv[2], "off", p[8], "ptr", p[9], "ms", ms, "frac", round(2000 * 24883200 / (ms / 1e3) / 8e12, 4), "ck", p[7])
