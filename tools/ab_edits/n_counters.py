# narrow kernel instrumented copy: per complex, the counts output holds (stored-list toggles, lazy/apparent
# toggles, pivot searches, V entries scanned) instead of the pair counts; read by tools/cnt_run.py
#   bash tools/build_patched.sh cnt tools/ab_edits/n_counters.py && DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_cnt.so python tools/cnt_run.py
import sys
p = sys.argv[1] + '/betti_kernels.hip'
s = open(p).read()
def rep(o, n):
    global s
    assert s.count(o) == 1, o[:60]
    s = s.replace(o, n)
# counters: stored-list toggles, lazy/apparent toggles, pivot searches, V entries scanned (dims 1+2)
rep("    uint32_t err;\n", "    uint32_t err;\n    int c_st = 0, c_lz = 0, c_ps = 0, c_ve = 0;\n")
rep("for (int u = 0; u < cnt && ok; ++u) ok = v_toggle(dim, rl(w, u), v);",
    "for (int u = 0; u < cnt && ok; ++u) { ok = v_toggle(dim, rl(w, u), v); ++c_st; }")
rep("                        ok = v_toggle(dim, app, v);", "                        ok = v_toggle(dim, app, v); ++c_lz;")
rep("                            ok = v_toggle(dim, m & ~kLazyBit, v);", "                            ok = v_toggle(dim, m & ~kLazyBit, v); ++c_lz;")
rep("                    tau = uni64(v > 0 ? pivot_of_V(dim, v, tau) : kInf);",
    "                    ++c_ps; c_ve += v;\n                    tau = uni64(v > 0 ? pivot_of_V(dim, v, tau) : kInf);")
rep("at(bl.counts + 4 * gi, lane) = lane == 0 ? cx.n_d0 : (lane == 1 ? cx.n_inf0 : (lane == 2 ? cx.n_p1 : cx.n_p2));",
    "at(bl.counts + 4 * gi, lane) = lane == 0 ? cx.c_st : (lane == 1 ? cx.c_lz : (lane == 2 ? cx.c_ps : cx.c_ve));")
open(p, 'w').write(s)
