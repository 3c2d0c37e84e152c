import sys
p = sys.argv[1] + '/betti_wide.hip'
s = open(p).read()
o = "            const int i = 1 + (int)walk_ticket(&ctr[kWcRow]);\n            if (i >= n) break;\n"
assert s.count(o) == 1
s = s.replace(o, "            const int i = 1 + (int)walk_ticket(&ctr[kWcRow]);\n            if (i >= 0) break;\n")
open(p, 'w').write(s)
