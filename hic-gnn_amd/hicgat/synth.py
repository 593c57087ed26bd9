"""Synthetic Hi-C inputs for the benchmark configurations.

* contacts: a kept pair (i, j) gets c_ij = max(1, Poisson(lam / |i - j|)), lam = 1e3 (a kept pair
  is always an edge, so the density is exactly the keep rate);
* ``dense``:  every i != j kept (synth-2000: nnz = N^2 incl. self loops);
* ``density``: keep (i, j) with p = min(1, kappa / |i - j|), kappa calibrated so the expected
  off-diagonal density is the target (synth-20000 at 1 %);
* features: x = 0.1 * N(0, 1) float32 [N, 512].

Everything is generated per diagonal offset from ``numpy.random.default_rng(seed)``, so the same
seed gives the same graph on any host; only the kept upper-triangle pairs are materialised.
"""
import numpy as np


def calibrate_kappa(n, density):
    d = np.arange(1, n, dtype=np.float64)
    w = 2.0 * (n - d)
    target = density * n * (n - 1)
    lo, hi = 0.0, float(n)
    for _ in range(200):
        k = 0.5 * (lo + hi)
        if np.sum(w * np.minimum(1.0, k / d)) < target:
            lo = k
        else:
            hi = k
    return 0.5 * (lo + hi)


def contact_pairs(n, density=None, lam=1e3, seed=0):
    """Upper-triangle contacts: returns (i int64, j int64, count float64) with i < j."""
    rng = np.random.default_rng(seed)
    kappa = None if density is None else calibrate_kappa(n, density)
    ii, jj, cc = [], [], []
    for d in range(1, n):
        m = n - d
        if kappa is None or kappa >= d:
            keep = np.arange(m)
        else:
            k = rng.binomial(m, kappa / d)
            if k == 0:
                continue
            keep = np.sort(rng.choice(m, size=k, replace=False))
        ii.append(keep)
        jj.append(keep + d)
        cc.append(np.maximum(1.0, rng.poisson(lam / d, size=len(keep)).astype(np.float64)))
    return np.concatenate(ii), np.concatenate(jj), np.concatenate(cc)


def features(n, f=512, seed=0, scale=0.1):
    rng = np.random.default_rng(seed + 1)
    return (scale * rng.standard_normal((n, f))).astype(np.float32)


WORKLOADS = {
    "synth-2000": dict(n=2000, density=None),
    "synth-20000": dict(n=20000, density=0.01),
}


def dense_contacts(n, i, j, c, device="cpu", dtype=None):
    """Symmetric dense [n, n] float64 contact matrix (zero diagonal) built on ``device``."""
    import torch
    A = torch.zeros((n, n), dtype=torch.float64, device=device)
    ti = torch.as_tensor(i, device=device)
    tj = torch.as_tensor(j, device=device)
    tc = torch.as_tensor(c, dtype=torch.float64, device=device)
    A[ti, tj] = tc
    A[tj, ti] = tc
    return A
