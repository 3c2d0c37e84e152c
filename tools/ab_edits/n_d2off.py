# narrow kernel ablation: no dim-2 pass at all, no dim-1 reduction
import sys
p = sys.argv[1] + '/betti_kernels.hip'
s = open(p).read()
o = "                cx.reduce_serial(1, nna);\n"
assert s.count(o) == 1
s = s.replace(o, "                (void)nna;\n")
o = "            if (dim_max >= 2 && cx.err == 0) {\n                int nna = 0;\n"
assert s.count(o) == 1
s = s.replace(o, "            if (dim_max >= 2 && cx.err == 0 && n > 1000) {\n                int nna = 0;\n")
open(p, 'w').write(s)
