"""dgn_dev_graph_betti (graph emit + Betti pass after one dgn_dev_graph_count, sharing the neighbour
count when the cutoffs agree) vs the separate calls: every output byte-identical, and the Betti
features against verbatim Ripser on a few atoms."""
import numpy as np
import pytest
import torch

import dgn
import oracle_py as O
from dgn import abi
from dgn.shard import Shard

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graph_rc,betti_rc", [(5.0, 5.0), (5.0, 4.5)])
def test_fused_equals_separate(ctx, graph_rc, betti_rc):
    dev = torch.device("cuda", 0)
    gp = abi.graph_params(r_cutoff=graph_rc, max_neighbors=20, rbf_cutoff=graph_rc, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    nb = abi.lib().dgn_rbf_bins(graph_rc, 0.1)
    out = []
    for fused in (False, True):
        sh = Shard(dgn, abi, "fcc", 4, 12, 3, dev)
        sh.alloc_graph(ctx, gp, nb, torch.float32)
        sh.alloc_betti()
        sh.step(ctx, gp, betti_rc, fused=fused)
        ctx.synchronize()
        out.append(sh.results())
    a, b = out
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    host = dgn.synth_batch("fcc", 4, 12, first_id=3 * 12)
    atoms = [0, 300, 1000]
    n = 256
    for gi in atoms:
        s = gi // n
        fo, co = O.ref_atom_betti(host["lattice"][s], host["positions"][s * n:(s + 1) * n],
                                  host["species"][s * n:(s + 1) * n], betti_rc, [gi - s * n])
        assert np.array_equal(b["counts"][gi], co[0])
        np.testing.assert_allclose(b["feat"][gi], fo[0], rtol=1e-6, atol=1e-12)
