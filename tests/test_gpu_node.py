"""Node features + topological block on the GPU through the C ABI:
species-keyed embedding gather (crystal_graph.cpp:19-21, bit-exact), PCA::transform of the Betti
statistics (pca.cpp:36-44, (x - mean) * components in f64; summation order differs from the CPU
product, tolerance 1e-12 relative to the row scale) and the N x (D + k) concatenation
(crystal_graph.cpp:65-67)."""
import numpy as np
import pytest

import dgn

pytestmark = pytest.mark.gpu


def _setup(torch, ctx, B=2, D=92, k=6):
    host = dgn.synth_batch("fcc", 4, B)
    dev = torch.device("cuda", 0)
    batch = {kk: torch.from_numpy(v).to(dev) for kk, v in host.items()}
    A = host["positions"].shape[0]
    S = int(host["species"].max()) + 2
    rng = np.random.default_rng(3)
    embed = rng.normal(size=(S, D))
    feat = torch.empty((A, 35), dtype=torch.float64, device=dev)
    ctx.dev_betti(batch, 5.0, feat)
    f = feat.cpu().numpy()
    mean = f.mean(axis=0)
    _, _, vt = np.linalg.svd(f - mean, full_matrices=False)
    comp = np.ascontiguousarray(vt[:k].T)  # 35 x k, row-major
    return host, batch, embed, feat, f, mean, comp, dev


def test_node_features_gather_pca_concat(ctx):
    import torch
    host, batch, embed, feat, f, mean, comp, dev = _setup(torch, ctx)
    A, D, k = f.shape[0], embed.shape[1], comp.shape[1]
    out = torch.empty((A, D + k), dtype=torch.float64, device=dev)
    ctx.dev_node_features(batch, torch.from_numpy(embed).to(dev), feat, torch.from_numpy(mean).to(dev),
                          torch.from_numpy(comp).to(dev), out)
    ctx.synchronize()
    o = out.cpu().numpy()
    assert np.array_equal(o[:, :D], embed[host["species"]])
    ref = (f - mean) @ comp
    scale = np.abs(f - mean).sum(axis=1, keepdims=True) * np.abs(comp).max() + 1e-300
    assert np.all(np.abs(o[:, D:] - ref) <= 1e-12 * scale)


def test_node_features_embedding_only(ctx):
    import torch
    host = dgn.synth_batch("sc", 4, 3)
    dev = torch.device("cuda", 0)
    batch = {kk: torch.from_numpy(v).to(dev) for kk, v in host.items()}
    S = int(host["species"].max()) + 1
    embed = np.arange(S * 4, dtype=np.float64).reshape(S, 4)
    out = torch.empty((host["positions"].shape[0], 4), dtype=torch.float64, device=dev)
    ctx.dev_node_features(batch, torch.from_numpy(embed).to(dev), None, None, None, out)
    assert np.array_equal(out.cpu().numpy(), embed[host["species"]])


def test_node_features_unknown_species_raises(ctx):
    import torch
    host = dgn.synth_batch("sc", 4, 1)
    dev = torch.device("cuda", 0)
    batch = {kk: torch.from_numpy(v).to(dev) for kk, v in host.items()}
    S = int(host["species"].max())  # one key short: the largest species has no row
    embed = torch.zeros((max(S, 1), 3), dtype=torch.float64, device=dev)
    out = torch.empty((host["positions"].shape[0], 3), dtype=torch.float64, device=dev)
    with pytest.raises(dgn.DgnError):
        ctx.dev_node_features(batch, embed, None, None, None, out)
