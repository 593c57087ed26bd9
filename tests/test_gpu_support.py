"""The fused loss over a truth in background + support form (hicgat_truth_support +
hicgat_pairdist_mse_fused_support) against the dense-truth kernel and an fp64 evaluation of the
reference's cdist -> MSELoss / pearsonr (models.py:661, HiC-GNN_main.py:127,
HiC_GAT_generalize_directly.py:210-225).  The two forms add the same terms in a different order
(bulk at the background value, then the support's difference), so values agree to fp32 / fp64
reassociation: moments 1e-6 relative, gradients 1e-5 of their max."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _contacts_truth(n, density, seed):
    import hicgat
    from hicgat import synth
    i, j, c = synth.contact_pairs(n, density=density, seed=seed)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    return A, hicgat.Truth.from_contacts(A, 0.5)


def _both(tr, coords, kind):
    import hicgat
    K = hicgat.kernels.default()
    n = tr.n
    out = {}
    for form in ("dense", "support"):
        stats = torch.empty(12, dtype=torch.float64, device=DEV)
        loss = torch.empty((), dtype=torch.float32, device=DEV)
        dc = torch.empty_like(coords)
        if form == "dense":
            K.fused_loss(coords, tr.buf, n, kind, 0, -1, stats, loss, dc)
        else:
            K.fused_loss_support(coords, tr.support, n, kind, stats, loss, dc)
        torch.cuda.synchronize()
        out[form] = (stats.cpu().numpy(), float(loss), dc.cpu().numpy())
    return out


def test_support_form_is_the_dense_truth():
    """hicgat_truth_support: sorted CSR of the off-diagonal entries != 1 of cont2dist's target, its
    values bit-equal to the dense truth, the diagonal; within the contact set (zero contacts -> 1)."""
    n = 1500
    A, tr = _contacts_truth(n, 0.02, 3)
    sf = tr.support
    assert sf is not None and sf.background == 1.0
    T = tr.dense()
    mask = T != 1.0
    mask.fill_diagonal_(False)
    r, c = mask.nonzero(as_tuple=True)
    assert torch.equal(sf.rowptr[1:].long().cpu(), torch.bincount(r, minlength=n).cumsum(0).cpu())
    assert torch.equal(sf.col.long(), c)
    assert torch.equal(sf.val, T[r, c])
    assert torch.equal(sf.diag, torch.diagonal(T))
    contact = A != 0
    contact.fill_diagonal_(False)
    # the support is the contact set less the contacts at exactly the max distance (T = mx/mx = 1)
    assert not bool((mask & ~contact).any())
    assert bool((T[contact & ~mask] == 1.0).all())
    print(f"support nnz {sf.nnz} of {n * n} ({sf.nnz / n / n:.3%})")


@pytest.mark.parametrize("n", [2, 3, 127, 128, 129, 700, 2000])
@pytest.mark.parametrize("kind", [0, 1])
def test_support_loss_matches_dense_and_fp64(n, kind):
    A, tr = _contacts_truth(n, 0.05 if n > 3 else None, n)
    if n > 3:
        assert tr.support is not None
    else:   # tiny graphs are all contacts: force the form anyway
        from hicgat import graph
        tr.support = graph.SupportForm.build(tr, 1.0, max_fraction=1.0)
    rng = np.random.default_rng(n)
    c = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32), device=DEV)
    r = _both(tr, c, kind)
    (sd, ld, gd), (ss, ls, gs) = r["dense"], r["support"]
    # fp64 reference of the reference's loss (exact distances)
    cd = c.double().cpu().requires_grad_(True)
    D = torch.cdist(cd, cd, compute_mode="donot_use_mm_for_euclid_dist")
    Tt = tr.dense().double().cpu()
    mse = torch.nn.functional.mse_loss(D, Tt)
    mse.backward()
    m = float(mse.detach())
    print(f"n={n} kind={kind}: mse dense {sd[7]:.9g} support {ss[7]:.9g} fp64 {m:.9g}; "
          f"grad rel {_rel(gs, gd):.2e}")
    assert abs(ss[7] - m) <= 1e-5 * m and abs(ss[7] - sd[7]) <= 1e-6 * abs(sd[7])
    for k in (0, 6) if kind == 0 else range(7):
        assert abs(ss[k] - sd[k]) <= 1e-6 * max(abs(sd[k]), 1e-30) + 1e-9, (k, ss[k], sd[k])
    if kind == 1 and n > 2:   # r's cancellation amplifies the fp32 rounding of a few-pair sum
        assert abs(ss[8] - sd[8]) < (1e-6 if n >= 100 else 1e-5)
    assert _rel(gs, gd) < 1e-5
    assert _rel(gs, cd.grad.numpy()) < 1e-5


def test_support_all_background_and_asymmetric_source():
    """An empty support (every off-diagonal entry at the background) and a non-symmetric source
    (Truth folds it into the symmetric form first; the diagonal carries the constant)."""
    import hicgat
    n = 300
    rng = np.random.default_rng(7)
    t = np.ones((n, n))
    np.fill_diagonal(t, 0.0)
    tr = hicgat.Truth(torch.tensor(t, device=DEV))
    assert tr.support is not None and tr.support.nnz == 0
    c = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32), device=DEV)
    for kind in (0, 1):
        (sd, _, gd), (ss, _, gs) = _both(tr, c, kind).values()
        assert abs(ss[7] - sd[7]) <= 1e-6 * sd[7] and _rel(gs, gd) < 1e-5
    k = rng.integers(0, n, size=(2, 400))
    t[k[0], k[1]] = rng.random(400) * 3
    tr = hicgat.Truth(torch.tensor(t, device=DEV))
    assert tr.asymmetric_source and tr.support is not None
    (sd, _, gd), (ss, _, gs) = _both(tr, c, 0).values()
    assert abs(ss[7] - sd[7]) <= 1e-6 * sd[7] and _rel(gs, gd) < 1e-5


def test_dense_truth_keeps_the_dense_path():
    """A truth with most entries off the background (synth-2000 is all contacts) has no support
    form: the loss streams the dense truth."""
    _, tr = _contacts_truth(600, None, 1)
    assert tr.support is None


@pytest.mark.parametrize("n", [700, 2000])
@pytest.mark.parametrize("scale", [1e-2, 1e-3])
def test_support_pearson_with_collapsed_coordinates(n, scale):
    """The combined loss's Pearson r (stats[8]) when the predicted distances are far below the
    background distance 1 (coordinates at 0.01 / 0.001 of unit scale: early training or a collapsed
    model).  The background form sums d^2 directly (the round-5 form rebuilt it as
    sum (d - 1)^2 + (2 sum d - n), a difference of two ~n-sized terms in fp32 that would lose the
    variance here): r, the moments and the total against an fp64 evaluation of the same pairs, and
    against the dense-truth kernel."""
    from scipy.stats import pearsonr
    A, tr = _contacts_truth(n, 0.05, n + 1)
    assert tr.support is not None
    rng = np.random.default_rng(n)
    c = torch.tensor((scale * rng.standard_normal((n, 3))).astype(np.float32), device=DEV)
    r = _both(tr, c, 1)
    (sd, _, _), (ss, _, _) = r["dense"], r["support"]
    cd = c.double().cpu()
    D = torch.cdist(cd, cd, compute_mode="donot_use_mm_for_euclid_dist")
    iu = np.triu_indices(n, 1)
    d = D.numpy()[iu]
    t = tr.dense().double().cpu().numpy()[iu]
    r64 = float(pearsonr(t, d)[0])
    sdd64 = float(np.sum(d * d))
    print(f"n={n} scale={scale}: r support {ss[8]:.9g} dense {sd[8]:.9g} fp64 {r64:.9g}; "
          f"sum d^2 support {ss[2]:.9g} fp64 {sdd64:.9g}")
    assert abs(ss[2] - sdd64) <= 1e-5 * sdd64
    assert abs(ss[8] - r64) <= 1e-5 and abs(sd[8] - r64) <= 1e-5
