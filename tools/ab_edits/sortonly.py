import sys
p = sys.argv[1] + '/betti_wide.hip'
s = open(p).read()
o = "        nna = sort_na(base, nna, dim == 2);\n"
assert s.count(o) == 1
s = s.replace(o, o + "        if (dim == 2) nna = 0;\n")
open(p, 'w').write(s)
