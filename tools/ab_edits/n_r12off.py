# narrow kernel ablation: no dim-1 and no dim-2 reduction (apparent passes kept)
import sys
p = sys.argv[1] + '/betti_kernels.hip'
s = open(p).read()
for o in ("                cx.reduce_serial(2, nna);\n", "                cx.reduce_serial(1, nna);\n"):
    assert s.count(o) == 1
    s = s.replace(o, "                (void)nna;\n")
open(p, 'w').write(s)
