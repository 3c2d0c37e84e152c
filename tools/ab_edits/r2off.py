import sys
p = sys.argv[1] + '/betti_wide.hip'
s = open(p).read()
o = "        if (err == 0u) reduce(2, nna2, base2);"
assert s.count(o) == 1
s = s.replace(o, "        (void)base2;")
open(p, 'w').write(s)
