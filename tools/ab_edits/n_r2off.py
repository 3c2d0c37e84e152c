# narrow kernel ablation: no dim-2 reduction (apparent pass kept)
import sys
p = sys.argv[1] + '/betti_kernels.hip'
s = open(p).read()
o = "                cx.reduce_serial(2, nna);\n"
assert s.count(o) == 1
s = s.replace(o, "                (void)nna;\n")
open(p, 'w').write(s)
