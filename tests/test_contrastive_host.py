"""CPU: the contrastive loss -- the oracle restatement and the host logic.

Reference: ``train_and_test_same_res_GAT_node2vec.py:107-134``: ``idx = triu_indices(n, n, 1)``,
``dist_truth = truth[idx]`` (truth = cont2dist(y, 1): float64), ``dist_out = cdist(coords)[idx]``
(float32), ``total = 0.0 + 0.1 * mean(|dist_truth - dist_out|)`` -- float64, differentiable.  No
fixture of the reference holds a contrastive run, so the oracle is pinned here to an independent
numpy evaluation of that formula and of its closed-form gradient, and the background + support
decomposition the kernels use (bulk at the background value + the contact set's corrections) to
the oracle through the CPU stand-in (tests/cpu_kernels.py, the contract of the HIP kernel).
"""
import numpy as np
import pytest
import torch


def _coords_truth(n, seed, sparse=True):
    from oracle import graph as ogr
    rng = np.random.default_rng(seed)
    if sparse:
        a = (rng.random((n, n)) < 0.06) * rng.integers(1, 40, (n, n)).astype(np.float64)
        a = np.triu(a, 1)
        a = a + a.T
        truth = ogr.cont2dist(torch.tensor(a), 1)
    else:
        t = rng.random((n, n))
        truth = torch.tensor((t + t.T) / 2)
        truth.fill_diagonal_(0)
    c = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32))
    return c, truth


@pytest.mark.parametrize("n,sparse", [(2, False), (7, False), (58, True), (300, True)])
def test_oracle_contrastive_matches_numpy_formula_and_gradient(n, sparse):
    from oracle import gat as og
    from oracle import loop as ol
    c, truth = _coords_truth(n, n, sparse)
    cr = c.clone().requires_grad_(True)
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        loss = ol.contrastive_loss(cr, truth)
        loss.backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    assert loss.dtype == torch.float64
    # numpy: float32 distances (the reference's cdist output dtype), float64 difference and mean
    cn = c.numpy().astype(np.float64)
    diff = cn[:, None, :] - cn[None, :, :]
    d32 = np.sqrt((diff ** 2).sum(-1)).astype(np.float32).astype(np.float64)
    iu = np.triu_indices(n, 1)
    r = d32[iu] - truth.numpy()[iu]
    # (torch forms the fp32 distance in fp32 arithmetic: 1-ulp differences, 1e-8 on the mean)
    assert abs(float(loss) - 0.1 * np.abs(r).mean()) <= 1e-7 * float(loss)
    # d total / d c_i = float32(0.1 / M) * sum_{j != i} sign(d_ij - t_ij) (c_i - c_j) / d_ij
    M = n * (n - 1) / 2
    s = np.zeros((n, n))
    s[iu] = np.sign(r)
    s = s + s.T
    with np.errstate(divide="ignore", invalid="ignore"):
        w = np.where(d32 > 0, s / d32, 0.0)
    g = float(np.float32(0.1 / M)) * (w[:, :, None] * diff).sum(1)
    assert np.max(np.abs(cr.grad.numpy() - g)) <= 1e-5 * max(np.max(np.abs(g)), 1e-30)


@pytest.mark.parametrize("n", [40, 300])
def test_background_support_decomposition_matches_oracle(n):
    """The kernels' form of the contrastive loss over cont2dist's target: every pair at the
    background value 1 (bulk tiles), plus per contact (support) entry the change |d - t| - |d - 1|
    and (sgn(d - t) - sgn(d - 1)) / d (c_i - c_j) -- in fp64 through the CPU stand-in of the kernel
    contract (tests/cpu_kernels.py), against the oracle's autograd."""
    import hicgat
    from cpu_kernels import CpuKernels
    from hicgat.graph import SupportForm
    from oracle import gat as og
    from oracle import loop as ol
    c, truth = _coords_truth(n, 11)
    tr = hicgat.Truth(truth.float())
    sf = SupportForm.build_host(tr, 1.0)
    K = CpuKernels()
    stats = torch.zeros(12, dtype=torch.float64)
    loss = torch.zeros(())
    dc = torch.zeros((n, 3))
    K.fused_loss_support_range(c, sf, n, 2, 0, K.num_tiles(n), 0, n, stats, loss, dc)
    cr = c.clone().requires_grad_(True)
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        ref = ol.contrastive_loss(cr, truth.float().double())     # the truth as the kernel stores it (fp32)
        ref.backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    assert abs(float(stats[10]) - float(ref)) <= 1e-7 * float(ref)     # fp64 vs fp32 distances
    assert float((dc - cr.grad).abs().max()) <= 1e-5 * float(cr.grad.abs().max())


def test_truth_upper_keeps_the_upper_triangle_as_given():
    """An asymmetric target (R's KR scaling rounds (x_i A_ij) x_j and (x_j A_ji) x_i apart): the MSE
    sees the symmetrised form (graph.Truth), the contrastive loss reads truth[triu] itself --
    ``Truth.upper()`` holds that triangle in both halves; a symmetric target is its own upper()."""
    import hicgat
    rng = np.random.default_rng(0)
    t = rng.random((9, 9)).astype(np.float32)
    tr = hicgat.Truth(torch.tensor(t))
    assert tr.asymmetric_source
    u = tr.upper().dense().numpy()
    iu = np.triu_indices(9, 1)
    assert np.array_equal(u[iu], t[iu]) and np.array_equal(u, u.T) and np.all(np.diag(u) == 0)
    s = hicgat.Truth(torch.tensor((t + t.T) / 2))
    assert s.upper() is s


def test_loss_kind_codes_match_the_header():
    import os
    import re
    from hicgat import ops
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "include", "hicgat.h")) as fh:
        h = fh.read()
    codes = dict((k.lower(), int(v)) for k, v in re.findall(r"HICGAT_LOSS_(\w+) = (\d+)", h))
    assert codes == ops.LOSS_KINDS
