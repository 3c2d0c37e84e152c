"""Which inputs overflow the Betti kernels' workspace caps naturally (no forced retry)?
Prints, per case, whether the capacity-retry launch ran and the pair counts.
    python tools/retry_probe.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python"), os.path.join(ROOT, "oracle")]
import dgn  # noqa: E402
import oracle_py as O  # noqa: E402


def tri_from_matrix(M):
    n = M.shape[0]
    return np.array([M[i, j] for i in range(1, n) for j in range(i)], np.float32)


def run(ctx, name, lowers, npts, thr, maxp):
    ctx.retry_count()
    t0 = time.perf_counter()
    try:
        pairs, counts = ctx.host_persistence_lower(lowers, npts, maxp, thr, cap=1 << 16)
        st = "ok"
    except Exception as e:  # noqa: BLE001
        counts, st = None, str(e)[:120]
    dt = time.perf_counter() - t0
    print(f"{name:34s} retried={ctx.retry_count()} {dt:7.3f}s {st} "
          f"counts={None if counts is None else counts.tolist()[:3]}", flush=True)


def cloud_matrix(rng, kind, n):
    if kind == "uniform":
        M = rng.uniform(0.0, 1.0, (n, n))
    elif kind == "ties4":
        M = rng.integers(1, 5, (n, n)).astype(float)
    elif kind == "chain":
        M = np.abs(np.subtract.outer(np.arange(n), np.arange(n))) + rng.uniform(0, 0.3, (n, n))
    else:
        if kind == "circle":
            t = rng.uniform(0, 2 * np.pi, n)
            X = np.stack([np.cos(t), np.sin(t), 0.01 * rng.standard_normal(n)], 1)
        elif kind == "sphere":
            X = rng.standard_normal((n, 3))
            X /= np.linalg.norm(X, axis=1, keepdims=True)
        elif kind == "ball3d":
            X = rng.uniform(-1, 1, (n, 3))
        else:
            u, v = rng.uniform(0, 2 * np.pi, (2, n))
            X = np.stack([(2 + np.cos(v)) * np.cos(u), (2 + np.cos(v)) * np.sin(u), np.sin(v)], 1)
        M = np.sqrt(((X[:, None] - X[None]) ** 2).sum(-1))
    M = np.triu(M, 1)
    return M + M.T


def main():
    ctx = dgn.Context(0)
    rng = np.random.default_rng(5)
    which = sys.argv[1] if len(sys.argv) > 1 else "narrow"
    if which == "narrow":
        cases = [(n, k) for n in (48, 64) for k in ("uniform", "ties4", "chain", "circle", "sphere", "ball3d", "torus")]
    else:
        cases = [(n, k) for n, k in ((80, "sphere"), (100, "sphere"), (100, "circle"), (130, "sphere"), (160, "circle"),
                                     (70, "uniform"), (80, "uniform"))]
    for n, kind in cases:
        M = cloud_matrix(rng, kind, n)
        thr = float(M.max()) + 1.0  # clique
        run(ctx, f"n={n} {kind} clique", tri_from_matrix(M)[None], np.array([n], np.int32), thr, n)


if __name__ == "__main__":
    main()
