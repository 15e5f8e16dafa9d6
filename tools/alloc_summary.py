import sys
for l in open(sys.argv[1]):
    p = l.rstrip("\n").split("\t")
    if p[0] == "run":
        print("r%s buf%s %s %-6s %s frac %s" % (p[1], p[2], p[3], p[4], p[5], p[9]))
    else:
        print(l.rstrip())
