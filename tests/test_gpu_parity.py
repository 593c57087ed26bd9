"""GPU parity: every HIP kernel (through libhicgat.so's C ABI) against the CPU oracle / fixtures.

Tolerances (north star: coordinates and loss within 1e-5 relative fp32):
  * graph build (a3, a13): bit-exact; cont2dist (a12): bit-exact with IEEE sqrt, <= 1 ulp of the
    reference fixture at factor 0.5 (torch CPU float64 sqrt is MKL VML, not correctly rounded);
  * Adam (a10): bit-exact against the torch-CPU restatement;
  * GATConv forward output, coordinates, loss: rtol 1e-5 (plus a tiny atol for values near 0);
  * gradients: rtol 1e-4 relative to the tensor's max magnitude (fp32 reassociation over up to
    4e6 edges; the reference's own CPU thread count changes them by the same order).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hicgat  # noqa: F401  (fails loudly if libhicgat.so is missing)


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def _golden_graph(case):
    import hicgat
    g = load_golden(f"graph_{case}.npz")
    y = torch.tensor(g["matrix"], dtype=torch.float64, device=DEV)
    y.fill_diagonal_(0)
    adj = hicgat.Adj.from_dense_device(y)
    return g, y, adj


# ---------------------------------------------------------------- a13 / a3 / a12 (bit-exact)
@pytest.mark.parametrize("case", ["chr19_1mb", "chr19_500kb", "synth256"])
def test_csr_from_dense_bit_exact(case):
    from oracle import graph as og
    g, _, adj = _golden_graph(case)
    assert np.array_equal(adj.storage.rowptr().numpy(), g["rowptr"])
    assert np.array_equal(adj.storage.col().numpy(), g["col"])
    rp, c = og.set_diag(g["rowptr"], g["col"])
    assert np.array_equal(adj.rowptr32.cpu().numpy(), rp)
    assert np.array_equal(adj.col32.cpu().numpy(), c)


def test_csr_from_dense_asymmetric_and_isolated():
    import hicgat
    from oracle import graph as og
    rng = np.random.default_rng(3)
    n = 300
    a = np.where(rng.random((n, n)) < 0.05, rng.random((n, n)), 0.0)   # asymmetric pattern
    a[7, :] = 0
    a[:, 7] = 0                                                          # isolated node 7
    a[11, 12] = np.nan                                                   # NaN counts as an edge
    np.fill_diagonal(a, 0)
    adj = hicgat.Adj.from_dense_device(torch.tensor(a, device=DEV))
    rp, c, _ = og.csr_from_matrix(a)
    assert np.array_equal(adj.storage.rowptr().numpy(), rp)
    assert np.array_equal(adj.storage.col().numpy(), c)
    r2, c2 = og.set_diag(rp, c)
    assert np.array_equal(adj.rowptr32.cpu().numpy(), r2) and np.array_equal(adj.col32.cpu().numpy(), c2)
    assert adj.rowptr32[8].item() - adj.rowptr32[7].item() == 1                # self loop only


def _cont2dist_ieee(y, f):
    """utils.py:75-80 with IEEE-correctly-rounded float64 sqrt (numpy)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        d = 1.0 / y
        d = np.sqrt(d) if f == 0.5 else d ** f
    np.fill_diagonal(d, 0)
    m = np.max(np.nan_to_num(d, posinf=0))
    return np.nan_to_num(d, posinf=m) / m


@pytest.mark.parametrize("case", ["chr19_1mb", "chr19_500kb", "synth256"])
@pytest.mark.parametrize("factor,key", [(0.5, "truth05"), (1, "truth1")])
def test_cont2dist_bit_exact(case, factor, key):
    """factor 1: bit-exact with the reference fixture.  factor 0.5: bit-exact with IEEE sqrt, and
    within 2 float64 ulps of the fixture -- the reference's torch CPU sqrt on float64 goes through
    MKL VML (tensors above ~128 elements), which returns the correctly rounded value minus 1 ulp
    for ~0.7 % of inputs ('Oracle and parity')."""
    import hicgat
    g, y, _ = _golden_graph(case)
    t = hicgat.cont2dist(y, factor).cpu().numpy()
    ieee = _cont2dist_ieee(y.cpu().numpy(), factor)
    assert np.array_equal(t, ieee)
    ulps = np.abs(t.view(np.int64) - g[key].view(np.int64))
    if factor == 1:
        assert ulps.max() == 0
    else:   # 1 ulp from the entry's sqrt, 1 more from the max it is divided by
        assert ulps.max() <= 2 and (ulps > 0).mean() < 0.02
    tr = hicgat.Truth.from_contacts(y, factor)
    d32 = tr.dense().cpu().numpy()
    assert tr.ld % 128 == 0
    # convert_to_matrix's triu + tril(T, 1) is asymmetric when the list has lower-triangle entries;
    # the fused-loss target then holds the equivalent symmetric form (graph.Truth)
    asym = not bool(np.array_equal(g[key], g[key].T))
    assert tr.asymmetric_source == asym
    if not asym:
        assert np.array_equal(d32, ieee.astype(np.float32))
        assert np.abs(d32.view(np.int32) - g[key].astype(np.float32).view(np.int32)).max() <= 1
    else:
        t = ieee.astype(np.float32).astype(np.float64)
        sym = (t + t.T) / 2
        np.fill_diagonal(sym, np.sqrt(np.diag(t) ** 2 + 0.5 * np.triu((t - t.T) ** 2, 1).sum(1)))
        np.testing.assert_allclose(d32, sym, rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------- GATConv (a2, a4, a5 + bwd)
def _random_graph(n, p, seed):
    rng = np.random.default_rng(seed)
    a = (rng.random((n, n)) < p).astype(np.float64)
    a = np.triu(a, 1)
    return a + a.T


def _gat_pair(seed=0, heads=2, out=256, fin=512):
    import hicgat
    from oracle import gat as og
    torch.manual_seed(seed)
    ref = og.GATConv(fin, out, heads=heads)
    torch.manual_seed(seed)
    mine = hicgat.GATConv(fin, out, heads=heads)
    for (k1, v1), (k2, v2) in zip(ref.state_dict().items(), mine.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2)
    with torch.no_grad():
        mine.bias.copy_(torch.randn_like(mine.bias) * 0.1)
        ref.bias.copy_(mine.bias)
    return ref, mine.to(DEV)


@pytest.mark.parametrize("n,p", [(58, 1.0), (130, 0.3), (257, 0.02), (600, 0.5)])
def test_gatconv_forward_backward_matches_oracle(n, p):
    import hicgat
    a = _random_graph(n, p, n)
    if n == 257:
        a[5, :] = 0
        a[:, 5] = 0                      # isolated node: row = self loop only
    ref, mine = _gat_pair(seed=n)
    adj = hicgat.Adj.from_dense_device(torch.tensor(a, device=DEV))
    rng = np.random.default_rng(n)
    x = torch.tensor((0.1 * rng.standard_normal((n, 512))).astype(np.float32))
    g = torch.tensor(rng.standard_normal((n, 512)).astype(np.float32))
    xr = x.clone().requires_grad_(True)
    out_r = ref(xr, (adj.storage.rowptr(), adj.storage.col()))
    (out_r * g).sum().backward()
    xm = x.to(DEV).requires_grad_(True)
    out_m = mine(xm, adj)
    (out_m * g.to(DEV)).sum().backward()
    np.testing.assert_allclose(out_m.detach().cpu().numpy(), out_r.detach().numpy(), rtol=1e-5, atol=1e-6)
    assert _rel(xm.grad.cpu(), xr.grad) < 1e-4
    for (name, pr), (_, pm) in zip(ref.named_parameters(), mine.named_parameters()):
        assert _rel(pm.grad.cpu(), pr.grad) < 1e-4, name


@pytest.mark.parametrize("n,p", [(58, 1.0), (257, 0.02), (600, 0.5)])
def test_gatconv_fused_relu_matches_oracle(n, p):
    """GATConv(x, act="relu") == relu(GATConv(x)) of the oracle, forward and backward (the relu
    of models.py:637 in the aggregation epilogue, its backward in the gather-free row pass)."""
    import hicgat
    a = _random_graph(n, p, n + 1)
    ref, mine = _gat_pair(seed=n + 1)
    adj = hicgat.Adj.from_dense_device(torch.tensor(a, device=DEV))
    rng = np.random.default_rng(n)
    x = torch.tensor((0.1 * rng.standard_normal((n, 512))).astype(np.float32))
    g = torch.tensor(rng.standard_normal((n, 512)).astype(np.float32))
    xr = x.clone().requires_grad_(True)
    out_r = torch.relu(ref(xr, (adj.storage.rowptr(), adj.storage.col())))
    (out_r * g).sum().backward()
    xm = x.to(DEV).requires_grad_(True)
    out_m = mine(xm, adj, act="relu")
    (out_m * g.to(DEV)).sum().backward()
    np.testing.assert_allclose(out_m.detach().cpu().numpy(), out_r.detach().numpy(), rtol=1e-5, atol=1e-6)
    assert _rel(xm.grad.cpu(), xr.grad) < 1e-4
    for (name, pr), (_, pm) in zip(ref.named_parameters(), mine.named_parameters()):
        assert _rel(pm.grad.cpu(), pr.grad) < 1e-4, name
    with torch.no_grad():                     # inference form (no out2) gives the same output
        assert torch.equal(mine(x.to(DEV), adj, act="relu"), out_m.detach())


@pytest.mark.parametrize("act", [0, 1])
def test_bwd_rows_equals_gather_dst(act):
    """The gather-free destination pass (delta = <dout, out - bias>, da_dst = <dout, out2> -
    delta S3) equals the gathering pass (per-edge <dout_i, h_j>) on the same inputs."""
    import hicgat
    from hicgat import synth
    K = hicgat.kernels.default()
    n = 3000
    i, j, c = synth.contact_pairs(n, density=0.03, seed=7)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    torch.manual_seed(3)
    h = torch.randn(n, 512, device=DEV) * 0.1
    a_s = torch.randn(n, 2, device=DEV)
    a_d = torch.randn(n, 2, device=DEV)
    b = torch.randn(512, device=DEV) * 0.1
    out = torch.empty(n, 512, device=DEV)
    out2 = torch.empty(n, 512, device=DEV)
    rs = torch.empty(n, 8, device=DEV)
    K.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, act, out, out2, rs)
    out_plain = torch.empty_like(out)
    rs_plain = torch.empty_like(rs)
    K.agg_fwd(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, out_plain, rs_plain)
    assert torch.equal(out, torch.relu(out_plain) if act else out_plain)
    assert torch.equal(rs[:, :4], rs_plain[:, :4])
    g = torch.randn(n, 512, device=DEV)
    dout = torch.empty_like(g)
    K.agg_bwd_rows(0, n, act, g, out, b, out2, dout, rs)
    dref = torch.where(out_plain > 0, g, torch.zeros_like(g)) if act else g
    if act:
        assert torch.equal(dout, dref)
    K.agg_bwd_dst(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, dref, 0.2, rs_plain)
    for k in (4, 5, 6, 7):
        assert _rel(rs[:, k].cpu(), rs_plain[:, k].cpu()) < 2e-5, k


def test_gat_linear_att_matches_torch():
    import hicgat
    from hicgat import _lib
    lib = _lib.lib()
    torch.manual_seed(1)
    for n in (1, 63, 64, 65, 1000):
        x = torch.randn(n, 512, device=DEV)
        W = torch.randn(512, 512, device=DEV) * 0.05
        al = torch.randn(1, 2, 256, device=DEV)
        ar = torch.randn(1, 2, 256, device=DEV)
        h = torch.empty(n, 512, device=DEV)
        a_s = torch.empty(n, 2, device=DEV)
        a_d = torch.empty(n, 2, device=DEV)
        _lib.check(lib.hicgat_gat_linear_att(_lib.ptr(x), _lib.ptr(W), _lib.ptr(al), _lib.ptr(ar), n, 512, 2,
                                             256, _lib.ptr(h), _lib.ptr(a_s), _lib.ptr(a_d), _lib.stream()), "lin")
        href = (x.double() @ W.double().t())
        assert _rel(h.cpu(), href.cpu()) < 2e-6
        hs = href.view(n, 2, 256)
        assert _rel(a_s.cpu(), (hs * al.double()).sum(-1).cpu()) < 1e-5
        assert _rel(a_d.cpu(), (hs * ar.double()).sum(-1).cpu()) < 1e-5
    assert hicgat  # silence


def test_gat_agg_long_rows_and_softmax_extremes():
    """Rows far longer than a wave chunk (2000 neighbours, not a multiple of 8) and logits with a
    large spread (the max subtraction must keep exp finite)."""
    import hicgat
    n = 2003
    a = np.ones((n, n)) - np.eye(n)
    ref, mine = _gat_pair(seed=5)
    with torch.no_grad():
        ref.att_l.mul_(40.0)
        mine.att_l.copy_(ref.att_l.to(DEV))
    adj = hicgat.Adj.from_dense_device(torch.tensor(a, device=DEV))
    x = torch.tensor((0.1 * np.random.default_rng(0).standard_normal((n, 512))).astype(np.float32))
    out_r = ref(x, (adj.storage.rowptr(), adj.storage.col()))
    out_m = mine(x.to(DEV), adj)
    np.testing.assert_allclose(out_m.detach().cpu().numpy(), out_r.detach().numpy(), rtol=1e-5, atol=2e-6)
    assert torch.isfinite(out_m).all()


# ---------------------------------------------------------------- a6: GEMM family / Linear
@pytest.mark.parametrize("m,n,k", [(20000, 256, 512), (777, 3, 64), (130, 129, 7), (64, 512, 512), (5, 1, 1)])
def test_gemm_layouts_match_torch(m, n, k):
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV)
    w = torch.randn(n, k, device=DEV)
    b = torch.randn(n, device=DEV)
    y = K.gemm(0, 0, m, n, k, x, w, torch.empty(m, n, device=DEV), bias=b)
    assert _rel(y.cpu(), (x.double() @ w.double().t() + b.double()).cpu()) < 5e-6
    dy = torch.randn(m, n, device=DEV)
    dx = K.gemm(0, 1, m, k, n, dy, w, torch.empty(m, k, device=DEV))
    assert _rel(dx.cpu(), (dy.double() @ w.double()).cpu()) < 5e-6
    for splits in (1, 3, 64, 100):
        dw = K.gemm(1, 1, n, k, m, dy, x, torch.empty(n, k, device=DEV), splits=splits)
        # one fp32 fma chain of m/splits terms per element: error grows like sqrt(m/splits)
        tol = 5e-6 * max(1.0, (m / splits / 512) ** 0.5)
        assert _rel(dw.cpu(), (dy.double().t() @ x.double()).cpu()) < tol
    acc = torch.ones(n, k, device=DEV)
    K.gemm(1, 1, n, k, m, dy, x, acc, accumulate=True, splits=3)
    assert _rel(acc.cpu(), (dy.double().t() @ x.double() + 1).cpu()) < 5e-6
    db = K.colsum(dy, torch.empty(n, device=DEV))
    assert _rel(db.cpu(), dy.double().sum(0).cpu()) < 5e-6


@pytest.mark.parametrize("m,n,k", [(20001, 512, 512), (1601, 128, 48), (2000, 384, 16)])
def test_tall_gemm_edges_and_accumulate(m, n, k):
    """The 160x128 LDS-DMA kernel (gemm_tall.hip) on ragged row counts, both B layouts, bias and
    accumulate, against fp64."""
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV)
    w = torch.randn(n, k, device=DEV)
    b = torch.randn(n, device=DEV)
    y0 = torch.randn(m, n, device=DEV)
    y = K.gemm(0, 0, m, n, k, x, w, y0.clone(), bias=b, accumulate=True)
    assert _rel(y.cpu(), (x.double() @ w.double().t() + b.double() + y0.double()).cpu()) < 5e-6
    dy = torch.randn(m, n, device=DEV)
    dx = K.gemm(0, 1, m, k, n, dy, w, torch.empty(m, k, device=DEV))
    assert _rel(dx.cpu(), (dy.double() @ w.double()).cpu()) < 5e-6
    if n % 128 == 0 and k % 16 == 0:   # same numbers with the tall kernel's strided-row operands
        xs = torch.randn(m, k + 4, device=DEV)[:, 2:2 + k]
        ys = K.gemm(0, 0, m, n, k, xs, w, torch.empty(m, n, device=DEV), bias=b)
        assert _rel(ys.cpu(), (xs.double() @ w.double().t() + b.double()).cpu()) < 5e-6


@pytest.mark.parametrize("m,n,k", [(2701, 512, 512), (2479, 256, 512), (2701, 512, 256), (1601, 384, 272),
                                   (3001, 192, 512)])
def test_row_split_gemm_matches_fp64(m, n, k):
    """Node-row GEMMs of a rank's shard (kernels.row_splits: the 64x128 kernel split over K into
    slabs added in split order), both B layouts, into a column slice of a wider output (ldc > N), with
    bias and accumulate, against fp64; and against the unsplit kernel (splits=1) to fp32 rounding."""
    import hicgat
    from hicgat import kernels as hk
    K = hicgat.kernels.default()
    assert hk.row_splits(m, n, k) > 1 and hk.row_splits(m, k, n) >= 1
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV)
    w = torch.randn(n, k, device=DEV)
    b = torch.randn(n, device=DEV)
    big = torch.randn(m, n + 64, device=DEV)
    ref = x.double() @ w.double().t() + b.double() + big[:, 32:32 + n].double()
    out = big.clone()
    K.gemm(0, 0, m, n, k, x, w, out[:, 32:32 + n], bias=b, accumulate=True)
    assert _rel(out[:, 32:32 + n].cpu(), ref.cpu()) < 5e-6
    assert torch.equal(out[:, :32], big[:, :32]) and torch.equal(out[:, 32 + n:], big[:, 32 + n:])
    one = K.gemm(0, 0, m, n, k, x, w, torch.empty(m, n, device=DEV), bias=b, splits=1)
    spl = K.gemm(0, 0, m, n, k, x, w, torch.empty(m, n, device=DEV), bias=b)
    assert _rel(spl.cpu(), one.double().cpu()) < 5e-6
    dy = torch.randn(m, n, device=DEV)
    dx = K.gemm(0, 1, m, k, n, dy, w, torch.empty(m, k, device=DEV))
    assert _rel(dx.cpu(), (dy.double() @ w.double()).cpu()) < 5e-6


@pytest.mark.parametrize("m,n,k,splits", [(128, 128, 1001, 3), (512, 256, 17, 1), (256, 128, 20000, 1),
                                          (128, 384, 4099, 64), (512, 512, 20000, 32)])
def test_wgrad_ragged_strided(m, n, k, splits):
    """The split-K weight-gradient GEMM (gemm.hip) on K not a multiple of its 16-row stage, splits
    whose last stage is partial, row-strided operands, with and without the bias column sums and
    accumulate, vs fp64."""
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(m + n + k + splits)
    dy = torch.randn(k, m + 4, device=DEV)[:, :m]
    x = torch.randn(k, n + 8, device=DEV)[:, 4:4 + n]
    rW = dy.double().t() @ x.double()
    tol = 5e-6 * max(1.0, (k / splits / 512) ** 0.5)
    dW0, db0 = torch.randn(m, n, device=DEV), torch.randn(m, device=DEV)
    dW, db = dW0.clone(), db0.clone()
    K.wgrad(dy, x, dW, db, accumulate=True, splits=splits)
    assert _rel(dW.cpu(), (rW + dW0.double()).cpu()) < tol
    assert _rel(db.cpu(), (dy.double().sum(0) + db0.double()).cpu()) < tol
    dW2 = K.gemm(1, 1, m, n, k, dy, x, torch.empty(m, n, device=DEV), splits=splits)
    assert _rel(dW2.cpu(), rW.cpu()) < tol


@pytest.mark.parametrize("splits", [1, 7, 78])
def test_wgrad_bias_fold_matches_fp64(splits):
    """hicgat_gemm_wgrad: dW = dY^T X and db = column sums of dY from ONE split-K GEMM launch (the
    bias partials ride in the slab), accumulate on and off, against fp64."""
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(splits)
    for (mo, ni) in ((256, 512), (3, 64), (130, 96)):
        dy = torch.randn(20000, mo, device=DEV)
        x = torch.randn(20000, ni, device=DEV)
        dW = torch.randn(mo, ni, device=DEV)
        db = torch.randn(mo, device=DEV)
        rW = dy.double().t() @ x.double() + dW.double()
        rb = dy.double().sum(0) + db.double()
        K.wgrad(dy, x, dW, db, accumulate=True, splits=splits)
        tol = 5e-6 * max(1.0, (20000 / splits / 512) ** 0.5)
        assert _rel(dW.cpu(), rW.cpu()) < tol and _rel(db.cpu(), rb.cpu()) < tol, (mo, ni)
        K.wgrad(dy, x, dW, None, splits=splits)
        assert _rel(dW.cpu(), (dy.double().t() @ x.double()).cpu()) < tol


def test_linear_autograd_matches_torch():
    import hicgat
    torch.manual_seed(0)
    lin = torch.nn.Linear(512, 256).to(DEV)
    x = torch.randn(3001, 512, device=DEV, requires_grad=True)
    y = hicgat.ops.linear(x, lin.weight, lin.bias)
    g = torch.randn_like(y)
    (y * g).sum().backward()
    gx, gw, gb = x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()
    x.grad = None
    lin.zero_grad()
    (torch.nn.functional.linear(x.double(), lin.weight.double(), lin.bias.double()) * g.double()).sum().backward()
    assert _rel(gx.cpu(), x.grad.cpu()) < 5e-6
    assert _rel(gw.cpu(), lin.weight.grad.cpu()) < 5e-6
    assert _rel(gb.cpu(), lin.bias.grad.cpu()) < 5e-6


@pytest.mark.parametrize("w", [64, 128, 256])
@pytest.mark.parametrize("with_res", [True, False])
def test_ln_relu_res_and_dual_linear_match_torch(w, with_res):
    import hicgat
    torch.manual_seed(w)
    lin1 = torch.nn.Linear(2 * w, w).to(DEV)
    lin2 = torch.nn.Linear(2 * w, w).to(DEV)
    norm = torch.nn.LayerNorm(w).to(DEV)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.uniform_(-0.2, 0.2)
    x = torch.randn(5003, 2 * w, device=DEV, requires_grad=True)
    y, r = hicgat.ops.dual_linear(x, lin1, lin2)
    z = hicgat.ops.ln_relu_res(y, norm, r if with_res else None)
    g = torch.randn_like(z)
    (z * g).sum().backward()
    mine = [t.grad.clone() for t in (x, lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias)]
    for t in (x, lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias):
        t.grad = None
    zr = torch.relu(norm(lin1(x))) + (lin2(x) if with_res else 0)
    assert _rel(z.detach().cpu(), zr.detach().cpu()) < 2e-5
    (zr * g).sum().backward()
    ref = [t.grad for t in (x, lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias)]
    for i, (a, b) in enumerate(zip(mine, ref)):
        if not with_res and i in (3, 4):
            assert b is None or b.abs().max() == 0
            continue
        assert _rel(a.cpu(), b.cpu()) < 5e-5, i


# ---------------------------------------------------------------- a7-a9: distance + loss
@pytest.mark.parametrize("n", [1, 2, 58, 129, 300])
def test_pairdist_fwd_bwd_matches_torch(n):
    import hicgat
    torch.manual_seed(n)
    c = torch.randn(n, 3, dtype=torch.float64)
    g = torch.randn(n, n, dtype=torch.float64)
    cr = c.clone().requires_grad_(True)
    dr = torch.cdist(cr, cr, compute_mode="donot_use_mm_for_euclid_dist")
    (dr * g).sum().backward()
    cm = c.float().to(DEV).requires_grad_(True)
    dm = hicgat.ops.pairwise_dist(cm)
    (dm * g.float().to(DEV)).sum().backward()
    assert _rel(dm.detach().cpu(), dr.detach()) < 1e-6
    assert torch.all(torch.diagonal(dm) == 0)
    if n > 1:
        assert _rel(cm.grad.cpu(), cr.grad) < 1e-5


@pytest.mark.parametrize("n", [2, 58, 128, 129, 400])
@pytest.mark.parametrize("kind", ["mse", "combined"])
def test_fused_loss_matches_oracle(n, kind):
    import hicgat
    from oracle import loop as ol
    rng = np.random.default_rng(n)
    t = rng.random((n, n))
    t = (t + t.T) / 2
    np.fill_diagonal(t, 0)
    truth = torch.tensor(t, dtype=torch.float64)
    c = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32))
    cr = c.clone().requires_grad_(True)
    out = torch.cdist(cr.double(), cr.double(), compute_mode="donot_use_mm_for_euclid_dist")
    if kind == "mse":
        lr = ol.mse_loss(out.float(), truth)
    else:
        lr = torch.nn.functional.mse_loss(out, truth)   # fp64 value; grad of mse only
    lr.backward()
    tr = hicgat.Truth(truth.to(DEV))
    cm = c.to(DEV).requires_grad_(True)
    lm, stats = hicgat.ops.fused_dist_loss(cm, tr, kind)
    lm.backward()
    st = stats.cpu().numpy()
    mse_ref = float(torch.nn.functional.mse_loss(out.detach(), truth))
    assert abs(st[7] - mse_ref) <= 1e-5 * mse_ref
    if kind == "mse":   # the Pearson moments are only formed for the combined loss
        assert np.isnan(st[8]) and np.all(st[1:6] == 0)
    elif n > 2:
        r_ref = ol.pearson_r(c.double(), truth)
        assert abs(st[8] - r_ref) < 1e-6
        if kind == "combined":
            alpha = min(1.0, 0.1 + 1.0 / (float(np.float32(st[7])) + 1e-6))
            assert abs(st[9] - alpha) < 1e-12
            assert abs(lm.item() - (np.float32(st[7]) + alpha * (1 - r_ref))) < 1e-5
    assert _rel(cm.grad.cpu(), cr.grad) < 1e-5
    assert abs(cm.grad.sum(0)).max().item() < 1e-5 * max(cm.grad.abs().max().item(), 1e-30) * n


def test_fused_loss_tile_ranges_sum_to_whole():
    """The multi-GPU contract: disjoint tile ranges give stats/dcoords that add up to the full
    call (moments exactly up to fp64 reassociation, dcoords to fp32 rounding)."""
    import hicgat
    from hicgat import _lib
    n = 700
    rng = np.random.default_rng(0)
    t = rng.random((n, n))
    t = (t + t.T) / 2
    np.fill_diagonal(t, 0)
    tr = hicgat.Truth(torch.tensor(t, device=DEV))
    c = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32), device=DEV)
    tiles = _lib.load().hicgat_pairdist_num_tiles(n, 1)
    full_l, full_s = hicgat.ops.fused_dist_loss(c.clone().requires_grad_(True), tr)
    parts = [(0, tiles // 3), (tiles // 3, tiles // 2), (tiles // 2, tiles)]
    acc = torch.zeros(7, dtype=torch.float64)
    g = torch.zeros(n, 3)
    for b, e in parts:
        cc = c.clone().requires_grad_(True)
        l, s = hicgat.ops.fused_dist_loss(cc, tr, tile_range=(b, e))
        l.backward()
        acc += s[:7].cpu()
        g += cc.grad.cpu()
    assert torch.allclose(acc, full_s[:7].cpu(), rtol=1e-12)
    cf = c.clone().requires_grad_(True)
    hicgat.ops.fused_dist_loss(cf, tr)[0].backward()
    assert _rel(g, cf.grad.cpu()) < 1e-6


# ---------------------------------------------------------------- a10: Adam
def test_adam_bit_exact_vs_torch_cpu_restatement():
    import hicgat
    from oracle import loop as ol
    rng = np.random.default_rng(0)
    n = 100003
    p0 = rng.standard_normal(n).astype(np.float32)
    params = [torch.nn.Parameter(torch.tensor(p0, device=DEV))]
    opt = hicgat.FlatAdam(params, lr=1e-3)
    p, m, v = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for step in range(1, 8):
        g = rng.standard_normal(n).astype(np.float32)
        opt.grad[:n].copy_(torch.tensor(g))
        opt.step()
        p, m, v = ol.adam_reference_step(p, g, m, v, step)
        assert np.array_equal(params[0].detach().cpu().numpy(), p), step


@pytest.mark.parametrize("zero_calls", [1, 2])
def test_adam_device_step_count_paths_bit_exact(zero_calls):
    """The graph-replayable Adam (device step count, host-tabulated constants) on the two paths that
    advance the count here -- zero_grad's one-launch zero + count (hicgat_step_begin; a second
    zero_grad in the same step must not count twice) and Adam's own increment -- against the
    host-constant Adam and the CPU restatement, bit for bit.  (The xagg step's count in its first
    launch is covered by the sharded graph-replay-equals-eager tests in test_gpu_dist.py.)"""
    import hicgat
    from oracle import loop as ol
    rng = np.random.default_rng(1)
    n = 4099
    p0 = rng.standard_normal(n).astype(np.float32)
    opts = []
    for mode in ("host", "zero_grad", "adam_increment"):
        params = [torch.nn.Parameter(torch.tensor(p0, device=DEV))]
        opt = hicgat.FlatAdam(params, lr=1e-3)
        if mode != "host":
            opt.enable_device_step()
        opts.append((mode, opt, params))
    p, m, v = p0.copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for step in range(1, 6):
        g = rng.standard_normal(n).astype(np.float32)
        for mode, opt, _ in opts:
            if mode == "zero_grad":
                for _ in range(zero_calls):
                    opt.zero_grad()
                assert float(opt.grad.abs().max()) == 0.0
            opt.grad[:n].copy_(torch.tensor(g))
            opt.step()
            if mode != "host":
                assert int(opt.step_ctr.item()) == step, (mode, step)
        p, m, v = ol.adam_reference_step(p, g, m, v, step)
        for mode, _, params in opts:
            assert np.array_equal(params[0].detach().cpu().numpy(), p), (mode, step)


# ---------------------------------------------------------------- models vs reference fixtures
def _oracle_exact(name, fx, g):
    """The oracle model with the fixture's weights, distances by the exact formula."""
    from oracle import gat as og
    m = og.MODELS[name]()
    m.load_state_dict({k[len("state::"):]: torch.tensor(v) for k, v in fx.items() if k.startswith("state::")})
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        adj = (torch.tensor(g["rowptr"]), torch.tensor(g["col"]))
        out = m(torch.tensor(fx["x"]), adj)
        torch.nn.functional.mse_loss(out.float(), torch.tensor(g["truth05"]).float()).backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    return m


@pytest.mark.parametrize("name", ["GATNetSelectiveResidualsUpdated", "GATNetHeadsChanged3LayersLeakyReLUv2"])
def test_model_matches_reference_fixture(name):
    """Forward/backward of a reference model class (models.py) on chr19 1 mb, same weights.

    The reference's torch.cdist uses the mm formula for N > 25: its distances
    carry O(1e-4) absolute error, its MSE is off by ~5e-6 relative and its gradients carry noise
    (dense3.bias, exactly 0 by translation invariance, comes out O(1e-6)).  The HIP path computes
    distances exactly, so: coordinates are checked against the fixture at 1e-5; D, loss and
    gradients against the oracle with exact distances (tight) and the fixture's loss loosely."""
    import hicgat
    fx = load_golden(f"model_{name}.npz")
    g = load_golden("graph_chr19_1mb.npz")
    torch.manual_seed(0)
    model = hicgat.MODELS[name]()
    for k, v in model.state_dict().items():
        assert np.array_equal(v.numpy(), fx[f"state::{k}"]), k          # same init from the seed
    model = model.to(DEV)
    y = torch.tensor(g["matrix"], device=DEV)
    y.fill_diagonal_(0)
    adj = hicgat.Adj.from_dense_device(y)
    x = torch.tensor(fx["x"], device=DEV)
    coords = model.get_model(x, adj)
    np.testing.assert_allclose(coords.detach().cpu().numpy(), fx["coords"], rtol=1e-5, atol=1e-6)
    out = model(x, adj)
    c64 = torch.tensor(fx["coords"]).double()
    d_exact = torch.cdist(c64, c64, compute_mode="donot_use_mm_for_euclid_dist")
    np.testing.assert_allclose(out.detach().cpu().numpy(), d_exact.numpy(), rtol=1e-5, atol=1e-6)
    tr = hicgat.Truth.from_contacts(y, 0.5)
    loss, stats, _ = model.loss(x, adj, tr, "combined")
    t = torch.tensor(g["truth05"])
    mse_exact = float(torch.nn.functional.mse_loss(d_exact, t))
    assert abs(stats[7].item() - mse_exact) <= 1e-5 * mse_exact
    assert abs(stats[7].item() - float(fx["mse"])) <= 3e-5 * float(fx["mse"])
    iu = np.triu_indices(len(c64), 1)
    r_exact = np.corrcoef(d_exact.numpy()[iu], g["truth05"][iu])[0, 1]
    # Pearson of the ~0.005-sized initial distances against T ~ 0.5 is ill-conditioned (the raw
    # moments cancel ~60x): 1e-7 relative coordinate differences move r by a few 1e-6
    assert abs(stats[8].item() - r_exact) < 2e-5
    # the fixture's r and total are built on the mm-formula distances, which at these tiny initial
    # coordinates are noise-dominated (v2: D ~ 1e-4 with 6e-5 error): checked via r_exact only
    alpha = min(1.0, 0.1 + 1.0 / (float(np.float32(stats[7].item())) + 1e-6))
    assert abs(loss.item() - (np.float32(stats[7].item()) + alpha * (1 - r_exact))) < 3e-5
    ref = _oracle_exact(name, fx, g)
    model.zero_grad()
    lm, _, _ = model.loss(x, adj, tr, "mse")
    lm.backward()
    gscale = max(pr.grad.abs().max().item() for pr in ref.parameters())
    for (k, p), pr in zip(model.named_parameters(), ref.parameters()):
        if pr.grad.abs().max().item() < 1e-3 * gscale:
            # zero in exact arithmetic: the last bias by translation invariance, and (v2 at these
            # 0.1-scale inputs) every bias whose units keep one activation sign over all nodes,
            # which makes sum_i g_i = 0 propagate up the tail; both sides are fp32 noise
            assert p.grad.abs().max().item() < 1e-3 * gscale, k
            continue
        assert _rel(p.grad.cpu(), pr.grad) < 2e-4, k


def _oracle_states(ref, x, radj, truth, K):
    """The oracle loop (HiC-GNN_main.py:117-132, torch.optim.Adam lr 1e-3) with the parameters
    before every step, the step's loss and its gradients recorded."""
    from oracle import loop as ol
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    out = []
    threads = torch.get_num_threads()
    torch.set_num_threads(1)   # the 1-thread oracle run of _thread_spread, step for step
    try:
        for _ in range(K):
            opt.zero_grad()
            state = {k: p.detach().clone() for k, p in ref.named_parameters()}
            val = ol.mse_loss(ref(x, radj), truth)
            val.backward()
            out.append((state, float(val.item()), {k: p.grad.detach().clone() for k, p in ref.named_parameters()}))
            opt.step()
    finally:
        torch.set_num_threads(threads)
    return out


def _replay_on_device(model, data, tr, states):
    """Teacher forcing: load each recorded oracle state into the device model, run the device's
    forward + backward from it, and return the worst relative loss error and the worst gradient
    error (max |err| / max |oracle| per tensor; tensors whose oracle gradient is below 1e-3 of the
    step's largest are only checked to stay that small)."""
    import hicgat
    opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
    params = dict(model.named_parameters())
    assert set(params) == set(states[0][0])
    worst_l, worst_g = 0.0, 0.0
    for state, l_ref, g_ref in states:
        with torch.no_grad():
            for k, v in state.items():
                params[k].copy_(v)
        opt.zero_grad()
        val, _, _ = model.loss(data.x, data.edge_index, tr, "mse")
        val.backward()
        worst_l = max(worst_l, abs(val.item() - l_ref) / l_ref)
        gscale = max(float(g.abs().max()) for g in g_ref.values())
        for k, g in g_ref.items():
            gd = params[k].grad.detach().cpu()
            if float(g.abs().max()) < 1e-3 * gscale:
                assert float(gd.abs().max()) < 1e-3 * gscale, k
                continue
            worst_g = max(worst_g, _rel(gd, g))
    return worst_l, worst_g


def _thread_spread(make, x, radj, truth, K):
    """The oracle's own run-to-run spread: the same loop at 1, 2, 4 and 8 threads (summation order
    changes); per step, the largest relative distance to the 1-thread loss."""
    from oracle import loop as ol
    threads = torch.get_num_threads()
    hist = {}
    try:
        for th in (1, 2, 4, 8):
            torch.set_num_threads(th)
            torch.manual_seed(0)
            hist[th] = np.array(ol.train(make(), x, radj, truth, steps=K))
    finally:
        torch.set_num_threads(threads)
    return hist[1], np.max([np.abs(h - hist[1]) / hist[1] for h in hist.values()], axis=0)


def test_train_loop_tracks_oracle():
    """HiC-GNN_main.py loop, fixed K = 25 on chr19 1 mb, vs the oracle loop (exact distances).
    Two checks.  Teacher-forced: from every state the oracle visits, the device's loss (1e-5) and
    gradients (2e-4) match -- a backward or loss bug anywhere along the trajectory shows here, no
    chaos involved.  Free-running: the device curve stays within 2x the spread the CPU oracle shows (its running max, two steps ahead)
    between its own 1/2/4/8-thread runs (measured live; it reaches ~5e-2 by step 9, because Adam
    turns rounding-level gradient differences into lr-sized steps)."""
    import hicgat
    from oracle import gat as og
    fx = load_golden("train_GATNetSelectiveResidualsUpdated.npz")
    mfx = load_golden("model_GATNetSelectiveResidualsUpdated.npz")
    g = load_golden("graph_chr19_1mb.npz")
    K = int(fx["steps"])
    x_h, truth_h = torch.tensor(mfx["x"]), torch.tensor(g["truth05"])
    radj = (torch.tensor(g["rowptr"]), torch.tensor(g["col"]))
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        ref_hist, spread = _thread_spread(og.GATNetSelectiveResidualsUpdated, x_h, radj, truth_h, K)
        torch.manual_seed(0)
        states = _oracle_states(og.GATNetSelectiveResidualsUpdated(), x_h, radj, truth_h, K)
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    assert np.array_equal([s[1] for s in states], ref_hist)
    y = torch.tensor(g["matrix"], device=DEV)
    y.fill_diagonal_(0)
    data = hicgat.Data(x=torch.tensor(mfx["x"], device=DEV), edge_index=hicgat.Adj.from_dense_device(y), y=y)
    tr = hicgat.Truth.from_contacts(y, 0.5)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    _, hist = hicgat.train.train(model, data, tr, steps=K)
    rel = np.abs(np.array(hist) - ref_hist) / ref_hist
    wl, wg = _replay_on_device(model, data, tr, states)
    np.set_printoptions(precision=2, linewidth=200)
    print(f"teacher-forced over {K} states: loss rel {wl:.2e}, grad rel {wg:.2e}")
    print("free-running rel", rel)
    print("oracle spread   ", spread)
    assert wl < 1e-5 and wg < 2e-4, (wl, wg)
    assert rel[0] < 1e-5 and rel[1] < 1e-5, rel[:3]
    assert rel[2] < 1e-4, rel[:3]
    # the oracle's own envelope with two steps of lookahead: when the chaotic growth sets in shifts
    # by a step or two between rounding paths (measured: one device run at 3.6e-3 on step 6, where
    # the host's 1/2/4/8-thread spread was 1.3e-3 and reached 2.9e-3 / 4.1e-3 on steps 7 / 8)
    run_rel, run_spread = np.maximum.accumulate(rel), np.maximum.accumulate(spread)
    ahead = run_spread[np.minimum(np.arange(len(spread)) + 2, len(spread) - 1)]
    assert np.all(run_rel <= 2 * ahead + 1e-4), (rel, spread)


def test_graph_replay_equals_eager_steps():
    """hipGraph-captured training steps (device-side Adam step counter) give the same bits as the
    eager steps."""
    import hicgat
    from hicgat import synth
    n = 1500
    i, j, c = synth.contact_pairs(n, density=0.05, seed=1)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    x = torch.tensor(synth.features(n, seed=1), device=DEV)
    res = []
    for graphed in (False, True):
        torch.manual_seed(0)
        model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
        losses = []
        if graphed:
            step = hicgat.graphs.captured_train_step(model, opt, x, adj, tr, warmup=2)
            losses += [None, None]
            for _ in range(4):
                losses.append(float(step()[0]))
        else:
            for _ in range(6):
                losses.append(float(hicgat.train.train_step(model, opt, x, adj, tr)[0]))
        res.append((losses, opt.flat.clone()))
    (le, pe), (lg, pg) = res
    assert le[2:] == lg[2:]
    assert torch.equal(pe, pg)


def test_overlapped_param_grads_same_bits(monkeypatch):
    """Parameter gradients on the side stream (ops.overlapped_param_grads, the train_step default)
    give the same bits as the serial backward, eagerly and inside a captured step, when the side
    work is the same launches (one per item: SIDE_GROUPED off, the big dW held for lin_l's grouped
    launch).  With the default grouped side launch (one hicgat_param_grads_grouped launch, its own
    K split) the eager and captured steps are bit-equal to each other and within fp32 reassociation
    of the serial backward."""
    import hicgat
    from hicgat import ops, synth
    n = 1200
    i, j, c = synth.contact_pairs(n, density=0.05, seed=2)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    x = torch.tensor(synth.features(n, seed=2), device=DEV)

    def run(overlap, graphed, grouped, steps=4):
        monkeypatch.setattr(ops, "OVERLAP_DEFAULT", overlap)
        monkeypatch.setattr(ops, "SIDE_GROUPED", grouped)
        monkeypatch.setattr(ops, "BIG_GROUP", 0.0 if grouped else 5e9)
        torch.manual_seed(0)
        model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
        if graphed:
            step = hicgat.graphs.captured_train_step(model, opt, x, adj, tr, warmup=1)
            losses = [float(step()[0]) for _ in range(steps - 1)]
        else:
            losses = [float(hicgat.train.train_step(model, opt, x, adj, tr)[0]) for _ in range(steps)][1:]
        torch.cuda.synchronize()
        return losses, opt.flat.clone(), opt.grad.clone()

    (l0, p0, g0), (l1, p1, g1), (l2, p2, g2) = (run(False, False, False), run(True, False, False),
                                                run(True, True, False))
    assert l0 == l1 == l2
    assert torch.equal(p0, p1) and torch.equal(p0, p2)
    assert torch.equal(g0, g1) and torch.equal(g0, g2)
    (l3, p3, g3), (l4, p4, g4) = run(True, False, True), run(True, True, True)
    assert l3 == l4 and torch.equal(p3, p4) and torch.equal(g3, g4)
    # grouped vs per-item side launches: the first step's gradients (later steps' Adam updates turn
    # sign flips of near-zero gradient entries into whole-lr differences)
    (_, _, g5), (_, _, g6) = run(False, False, False, steps=1), run(True, False, True, steps=1)
    assert _rel(g6.cpu(), g5.cpu()) < 1e-5


def test_dscc_matches_scipy():
    import hicgat
    from scipy.stats import spearmanr
    g = load_golden("graph_chr19_500kb.npz")
    rng = np.random.default_rng(0)
    n = g["truth05"].shape[0]
    c = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32), device=DEV)
    t = torch.tensor(g["truth05"], device=DEV)
    rho = hicgat.metrics.dscc(c, t)
    iu = np.triu_indices(n, 1)
    d_gpu = hicgat.ops.pairwise_dist(c).cpu().numpy()
    assert abs(rho - spearmanr(g["truth05"][iu], d_gpu[iu])[0]) < 1e-12      # ranking logic, ties
    d = torch.cdist(c.cpu(), c.cpu(), compute_mode="donot_use_mm_for_euclid_dist").numpy()
    assert abs(rho - spearmanr(g["truth05"][iu], d[iu])[0]) < 1e-6           # 1-ulp sqrt ties


# ---------------------------------------------------------------- full-size properties
def test_full_size_synth20000_properties():
    """At BASELINE's N = 20000 / 1 % size: (i) 24 sampled rows of the GAT aggregation against an
    fp64 host evaluation of those rows, (ii) softmax weights sum to 1 (h == const rows give
    out == const + bias), (iii) translation invariance of the distance-loss gradient."""
    import hicgat
    from hicgat import _lib, synth
    n = 20000
    i, j, c = synth.contact_pairs(n, density=0.01, seed=0)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    nnz = adj.device_nnz
    assert abs((nnz - n) / (n * (n - 1)) - 0.01) < 2e-4
    torch.manual_seed(0)
    conv = hicgat.GATConv(512, 256, heads=2).to(DEV)
    x = torch.tensor(synth.features(n), device=DEV)
    with torch.no_grad():
        out = conv(x, adj)
        h = x.double() @ conv.lin_l.weight.double().t()
        hv = h.view(n, 2, 256)
        a_s = (hv * conv.att_l.double()).sum(-1)
        a_d = (hv * conv.att_r.double()).sum(-1)
        rp = adj.rowptr32.cpu().numpy()
        cl = adj.col32.cpu().numpy()
        for r in np.random.default_rng(1).choice(n, 24, replace=False):
            nb = torch.tensor(cl[rp[r]:rp[r + 1]].astype(np.int64), device=DEV)
            e = torch.nn.functional.leaky_relu(a_s[nb] + a_d[r], 0.2)
            al = torch.softmax(e, 0)
            ref = (al.unsqueeze(-1) * hv[nb]).sum(0).reshape(-1) + conv.bias.double()
            assert _rel(out[r].cpu(), ref.cpu()) < 1e-5
    lib = _lib.lib()
    hconst = torch.full((n, 512), 0.75, device=DEV)
    a_s = torch.randn(n, 2, device=DEV)
    a_d = torch.randn(n, 2, device=DEV)
    bias = torch.randn(512, device=DEV)
    o = torch.empty(n, 512, device=DEV)
    rs = torch.empty(n, 8, device=DEV)
    _lib.check(lib.hicgat_gat_agg_fwd(_lib.ptr(adj.rowptr32), _lib.ptr(adj.col32), n, nnz, 2, 256, 0, n,
                                      _lib.ptr(hconst), _lib.ptr(a_s), _lib.ptr(a_d), _lib.ptr(bias), 0.2,
                                      _lib.ptr(o), _lib.ptr(rs), _lib.stream()), "agg")
    assert torch.allclose(o, 0.75 + bias.expand_as(o), rtol=0, atol=2e-6)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    cc = torch.randn(n, 3, device=DEV).requires_grad_(True)
    loss, stats = hicgat.ops.fused_dist_loss(cc, tr)
    loss.backward()
    gsum = cc.grad.double().sum(0).abs().max().item()
    assert gsum < 1e-4 * cc.grad.abs().max().item() * np.sqrt(n)
    assert np.isfinite(stats.cpu().numpy()[:8]).all()
    _, stats_c = hicgat.ops.fused_dist_loss(cc.detach(), tr, "combined")
    sc = stats_c.cpu().numpy()
    assert np.isfinite(sc[:11]).all() and -1 <= sc[8] <= 1
    s0 = stats.cpu().numpy()[0]
    assert abs(sc[0] - s0) <= 1e-12 * s0            # same sum (d - t)^2, Pearson on or off


# ---------------------------------------------------------------- f1: SAGEConv / Net baseline
@pytest.mark.parametrize("case", ["chr19_1mb", "chr19_500kb", "synth256"])
def test_sage_weights_bit_exact(case):
    """Device edge weights (networkx semantics) and 1/degree == the host derivation and oracle."""
    import hicgat
    from oracle import sage
    g, y, adj = _golden_graph(case)
    n = y.shape[0]
    assert np.array_equal(adj.storage.value().numpy(), g["value"])
    rp, c, v = (torch.tensor(g[k]) for k in ("rowptr", "col", "value"))
    r = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    host = hicgat.Adj(r, c, v, (n, n)).to("cpu")
    assert torch.equal(adj.value32.cpu(), host.value32)
    assert np.array_equal(adj.inv_deg.cpu().numpy(), sage.degree_inverse(g["rowptr"], g["col"], g["value"], n))


@pytest.mark.parametrize("n,p,F", [(58, 1.0, 512), (257, 0.05, 512), (1000, 0.1, 512), (130, 0.3, 100)])
def test_sage_agg_matches_oracle(n, p, F):
    import hicgat
    from oracle import graph as ogr
    from oracle import sage
    rng = np.random.default_rng(n)
    a = np.triu(np.where(rng.random((n, n)) < p, rng.integers(1, 1000, (n, n)).astype(np.float64), 0.0), 1)
    if n == 257:
        a[5, :] = 0
        a[:, 5] = 0                        # isolated node: inv_deg = inf, its row aggregates nothing
    a = a + a.T
    adj = hicgat.Adj.from_dense_device(torch.tensor(a, device=DEV))
    rp, c, v = ogr.csr_from_matrix(a)
    x = torch.tensor((1.5 * rng.standard_normal((n, F))).astype(np.float32))
    ref = sage.sage_aggregate(x, rp, c, v)
    K = hicgat.kernels.default()
    xd = x.to(DEV)
    z = torch.full((n, 2 * F), np.nan, device=DEV)
    K.sage_agg(adj.rowptr32, adj.col32, adj.value32, adj.inv_deg, 0, n, xd, z, write_trunc=True)
    np.testing.assert_allclose(z[:, :F].cpu().numpy(), ref.numpy(), rtol=1e-5, atol=1e-6 * ref.abs().max().item())
    assert torch.equal(z[:, F:].cpu(), x.long().float())
    # adjoint (d agg -> d x) against the oracle's autograd
    xr = x.clone().double().requires_grad_(True)
    gout = torch.tensor(rng.standard_normal((n, F)))
    (sage._SageAggFn.apply(xr, torch.tensor(rp), torch.tensor(c), torch.tensor(v)) * gout).sum().backward()
    dx = K.sage_agg(adj.rowptr32, adj.col32, adj.value32, adj.inv_deg, 0, n, gout.float().to(DEV),
                    torch.empty((n, F), device=DEV), transpose=True)
    assert _rel(dx.cpu(), xr.grad) < 1e-5
    # a row range writes only its rows
    z2 = torch.zeros((n, F), device=DEV)
    K.sage_agg(adj.rowptr32, adj.col32, adj.value32, adj.inv_deg, 3, n // 2, xd, z2)
    assert torch.equal(z2[3:n // 2], z[3:n // 2, :F]) and z2[:3].abs().sum() == 0 and z2[n // 2:].abs().sum() == 0


def test_net_matches_reference_fixture():
    """The baseline Net (models.py:14-55, layers.py SAGEConv) on chr19 1 mb vs the fixture
    recorded from the reference's code: coordinates 1e-5; D / MSE vs exact distances; gradients
    vs the oracle with exact distances."""
    import hicgat
    from oracle import gat as og
    from oracle import sage
    fx = load_golden("model_Net.npz")
    g, y, adj = _golden_graph("chr19_1mb")
    state = {k[len("state::"):]: torch.tensor(v) for k, v in fx.items() if k.startswith("state::")}
    model = hicgat.Net().to(DEV)
    model.load_state_dict(state)
    x = torch.tensor(fx["x"], device=DEV)
    coords = model.get_model(x, adj)
    np.testing.assert_allclose(coords.detach().cpu().numpy(), fx["coords"], rtol=1e-5,
                               atol=1e-5 * np.abs(fx["coords"]).max())
    out = model(x, adj)
    c64 = torch.tensor(fx["coords"]).double()
    d_exact = torch.cdist(c64, c64, compute_mode="donot_use_mm_for_euclid_dist")
    np.testing.assert_allclose(out.detach().cpu().numpy(), d_exact.numpy(), rtol=1e-5, atol=1e-5 * d_exact.max().item())
    tr = hicgat.Truth.from_contacts(y, 0.5)
    loss, stats, _ = model.loss(x, adj, tr, "mse")
    mse_exact = float(torch.nn.functional.mse_loss(d_exact, torch.tensor(g["truth05"])))
    assert abs(stats[7].item() - mse_exact) <= 2e-5 * mse_exact
    ref = sage.Net()
    ref.load_state_dict(state)
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        radj = (torch.tensor(g["rowptr"]), torch.tensor(g["col"]), torch.tensor(g["value"]))
        torch.nn.functional.mse_loss(ref(torch.tensor(fx["x"]), radj).float(),
                                     torch.tensor(g["truth05"]).float()).backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    model.zero_grad()
    loss.backward()
    gscale = max(p.grad.abs().max().item() for p in ref.parameters())
    for (k, p), pr in zip(model.named_parameters(), ref.parameters()):
        if pr.grad.abs().max().item() < 1e-3 * gscale:
            assert p.grad.abs().max().item() < 1e-3 * gscale, k
            continue
        assert _rel(p.grad.cpu(), pr.grad) < 2e-4, k


def test_net_train_loop_tracks_oracle():
    """HiC-GNN_main.py loop with the baseline Net (fixed K = 10) vs the oracle loop: teacher-forced
    loss / gradients from every oracle state, and the free-running curve (the CPU oracle is
    thread-count invariant here, measured: spread 0)."""
    import hicgat
    from oracle import gat as og
    from oracle import sage
    fx = load_golden("model_Net.npz")
    g, y, adj = _golden_graph("chr19_1mb")
    x_h, truth_h = torch.tensor(fx["x"]), torch.tensor(g["truth05"])
    radj = (torch.tensor(g["rowptr"]), torch.tensor(g["col"]), torch.tensor(g["value"]))
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        ref_hist, spread = _thread_spread(sage.Net, x_h, radj, truth_h, 10)
        torch.manual_seed(0)
        states = _oracle_states(sage.Net(), x_h, radj, truth_h, 10)
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    torch.manual_seed(0)
    model = hicgat.Net().to(DEV)
    data = hicgat.Data(x=torch.tensor(fx["x"], device=DEV), edge_index=adj, y=y)
    tr = hicgat.Truth.from_contacts(y, 0.5)
    _, hist = hicgat.train.train(model, data, tr, steps=10)
    rel = np.abs(np.array(hist) - ref_hist) / ref_hist
    wl, wg = _replay_on_device(model, data, tr, states)
    np.set_printoptions(precision=2, linewidth=200)
    print(f"teacher-forced over 10 states: loss rel {wl:.2e}, grad rel {wg:.2e}; free-running rel {rel}; "
          f"oracle spread {spread}")
    assert wl < 1e-5 and wg < 2e-4, (wl, wg)
    assert rel[0] < 1e-5 and rel[1] < 1e-4, rel[:3]
    assert np.all(rel < 0.05), rel


@pytest.mark.parametrize("K,N", [(0, 5), (1, 3), (64, 64), (65, 100), (5000, 3), (20000, 512), (1024, 512),
                                 (40, 300000)])
def test_colsum_deterministic_column_sums(K, N):
    """The fixed-order column reduction (bias / LayerNorm / split-K sums): tall multi-pass, wide
    one-pass, empty, accumulate; bitwise repeatable."""
    import hicgat
    K_ = hicgat.kernels.default()
    torch.manual_seed(K + N)
    A = torch.randn(K, N, device=DEV)
    out = K_.colsum(A, torch.full((N,), np.nan, device=DEV))
    ref = A.double().sum(0)
    assert _rel(out.cpu(), ref.cpu()) < 1e-5 if K else torch.all(out == 0)
    again = K_.colsum(A, torch.empty(N, device=DEV))
    assert torch.equal(out, again)
    base = torch.randn(N, device=DEV)
    acc = K_.colsum(A, base.clone(), accumulate=True)
    assert _rel(acc.cpu(), (ref + base.double()).cpu()) < 1e-5
    if K > 64:   # strided rows (lda > N)
        B = torch.randn(K, N + 7, device=DEV)[:, 3:3 + N]
        assert _rel(K_.colsum(B, torch.empty(N, device=DEV)).cpu(), B.double().sum(0).cpu()) < 1e-5


@pytest.mark.parametrize("order", ["parameters", "flat"])
@pytest.mark.parametrize("name", ["GATNetSelectiveResidualsUpdated", "GATNetHeadsChanged3LayersLeakyReLUv2", "Net"])
def test_grad_sink_equals_autograd_accumulation(name, order):
    """With FlatAdam attached, the backward kernels add parameter gradients straight into the flat
    buffer (no autograd add); the result is bitwise the ordinary autograd gradient, and a torch
    ``model.zero_grad()`` (set_to_none) in between is folded back by FlatAdam."""
    import hicgat
    from hicgat import synth
    n = 700
    i, j, c = synth.contact_pairs(n, density=0.05, seed=3)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    x = torch.tensor(synth.features(n, seed=3), device=DEV)
    torch.manual_seed(0)
    m1 = hicgat.MODELS[name]().to(DEV)
    torch.manual_seed(0)
    m2 = hicgat.MODELS[name]().to(DEV)
    params = m1.flat_parameters() if order == "flat" else m1.parameters()
    opt = hicgat.FlatAdam(params, lr=1e-3)
    assert {id(p) for p in opt.params} == {id(p) for p in m1.parameters()}
    opt.zero_grad()
    m1.loss(x, adj, tr)[0].backward()
    m2.loss(x, adj, tr)[0].backward()
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert p1.grad.data_ptr() >= opt.grad.data_ptr(), k            # still the flat-buffer view
        if order == "parameters":
            assert torch.equal(p1.grad, p2.grad), k
        else:   # adjacent pairs: one 2W-row dW GEMM / 2W-wide column sum (other split-K blocking)
            assert _rel(p1.grad.cpu(), p2.grad.cpu()) < 1e-5, k
    m1.zero_grad()                                                      # torch: grads -> None
    m1.loss(x, adj, tr)[0].backward()
    opt.step()
    g = opt.grad.clone()
    opt.zero_grad()
    m1.loss(x, adj, tr)[0].backward()
    assert g.abs().sum() > 0 and torch.all(opt.grad.abs().sum() > 0)


# ---------------------------------------------------------------- f2: KR normalisation on the GPU
def _kr_inputs():
    rng = np.random.default_rng(4)
    n = 600
    a = rng.random((n, n)) * (rng.random((n, n)) < 0.3) * 100
    a = np.triu(a, 1)
    a = a + a.T
    a[17, :] = 0
    a[:, 17] = 0
    a[40, 41] = a[41, 40] = np.nan
    return a


@pytest.mark.parametrize("case", ["chr19_1mb", "chr19_500kb", "synth600"])
def test_kr_device_matches_oracle(case):
    """hicgat.kr.KRnorm (HIP matvec / scale + device CG bookkeeping) vs the r_utils.R restatement:
    the same kept rows and NaN positions, values equal after the 6-digit rounding except where the
    two summation orders straddle a rounding boundary (one unit of 1e-6, rare)."""
    import hicgat
    from oracle import kr
    if case == "synth600":
        m = _kr_inputs()
    else:
        m = load_golden(f"graph_{case}.npz")["matrix"].copy()
        np.fill_diagonal(m, 0)
    ref, keep_r = kr.krnorm(m)
    out, keep, info = hicgat.kr.KRnorm(m, return_info=True)
    out = out.cpu().numpy()
    assert np.array_equal(keep.cpu().numpy(), keep_r)
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    ok = ~np.isnan(ref)
    diff = np.abs(out[ok] - ref[ok])
    assert diff.max() <= 1.0000001e-6
    assert (diff > 0).mean() < 0.01
    assert np.array_equal(out[ok], np.rint(out[ok] * 1e6) / 1e6)


@pytest.mark.parametrize("case,pdb,logged", [
    ("chr19_1mb", "GM12878_1mb_chr19_list_structure.pdb", 0.945986103111681),
    ("chr19_500kb", "GM12878_500kb_chr19_list_generalized_structure.pdb", 0.8074002899996215)])
def test_kr_device_reproduces_logged_dscc(case, pdb, logged):
    """Device KR -> device load_input / cont2dist(0.4) -> dSCC against the reference's PDB
    coordinates = the dSCC of the reference's log."""
    import os
    import hicgat
    from conftest import GOLDEN
    m = load_golden(f"graph_{case}.npz")["matrix"].copy()
    np.fill_diagonal(m, 0)
    normed, _ = hicgat.kr.KRnorm(m)
    data = hicgat.load_input(normed.cpu().numpy(), np.zeros((m.shape[0], 1), np.float32))
    t = hicgat.cont2dist(data.y, 0.4)
    c = torch.tensor(hicgat.io.read_pdb_coords(os.path.join(GOLDEN, pdb)), dtype=torch.float64)
    d = torch.cdist(c, c, compute_mode="donot_use_mm_for_euclid_dist").to(DEV)
    rho = hicgat.metrics.spearman(hicgat.metrics.triu_pairs(t), hicgat.metrics.triu_pairs(d))
    assert abs(rho - logged) < 3e-6


# ---------------------------------------------------------------- f3: Procrustes / generalisation
def test_domain_alignment_device_full_rank_matches_reference():
    """F = 32 < matched bins: the Procrustes rotation is unique -> the reference's fitembed."""
    import hicgat
    fx = load_golden("align_chr19_f32.npz")
    fit = hicgat.align.domain_alignment(fx["list1"], fx["list2"], fx["emb1"], fx["emb2"]).cpu().numpy()
    assert _rel(fit, fx["fitembed"]) < 2e-5


def test_domain_alignment_device_rank_deficient_is_a_procrustes_optimum():
    """F = 512 > matched bins (the real 1 mb -> 500 kb case): R is orthogonal and reaches the same
    optimum ||A R - B||_F as the reference's scipy solution (R itself is not unique there)."""
    import hicgat
    from oracle import align
    fx = load_golden("align_chr19_f512.npz")
    ia, ib = hicgat.align.matched_rows(fx["list1"], fx["list2"])
    ra, rb = align.matched_rows(fx["list1"], fx["list2"])
    assert np.array_equal(ia, ra) and np.array_equal(ib, rb)
    A = torch.tensor(fx["emb2"][ia], device=DEV)
    B = torch.tensor(fx["emb1"][ib], device=DEV)
    R = hicgat.align.procrustes(A, B).double()
    assert (R.t() @ R - torch.eye(512, dtype=torch.float64, device=DEV)).abs().max().item() < 1e-5
    _, Rr, Ar, Br = align.domain_alignment(fx["list1"], fx["list2"], fx["emb1"], fx["emb2"])
    obj = torch.linalg.norm(A.double() @ R - B.double()).item()
    obj_ref = np.linalg.norm(Ar.astype(np.float64) @ Rr.astype(np.float64) - Br)
    assert abs(obj - obj_ref) <= 1e-5 * obj_ref
    fit = hicgat.align.domain_alignment(fx["list1"], fx["list2"], fx["emb1"], fx["emb2"])
    assert _rel(fit.cpu(), (torch.tensor(fx["emb2"], device=DEV).double() @ R).cpu()) < 1e-5


def test_generalize_matches_oracle_pipeline():
    """HiC_GAT_generalize_directly.py:312-336 on chr19 500 kb: aligned embeddings -> load_input ->
    get_model -> dSCC vs cont2dist(normed, 1); the oracle model with the same weights on the same
    aligned embeddings gives the same dSCC."""
    import hicgat
    from scipy.stats import spearmanr
    from oracle import gat as og
    from oracle import graph as ogr
    from oracle import kr
    fx = load_golden("align_chr19_f512.npz")
    emb1 = (0.1 * fx["emb1"]).astype(np.float32)
    emb2 = (0.1 * fx["emb2"]).astype(np.float32)
    m = load_golden("graph_chr19_500kb.npz")["matrix"].copy()
    np.fill_diagonal(m, 0)
    normed, _ = kr.krnorm(m)
    torch.manual_seed(0)
    ref = og.GATNetSelectiveResidualsUpdated()
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    rho, coords = hicgat.align.generalize(model, fx["list1"], fx["list2"], emb1, emb2, normed, 1)
    fit = hicgat.align.domain_alignment(fx["list1"], fx["list2"], emb1, emb2).cpu()
    d = ogr.load_input(normed.copy(), fit.numpy())
    c_ref = ref.get_model(d["x"], (torch.tensor(d["rowptr"]), torch.tensor(d["col"]))).detach()
    np.testing.assert_allclose(coords.cpu().numpy(), c_ref.numpy(), rtol=1e-5, atol=1e-6)
    t = ogr.cont2dist(d["y"], 1).float().numpy()
    iu = np.triu_indices(len(t), 1)
    dd = torch.cdist(c_ref, c_ref, compute_mode="donot_use_mm_for_euclid_dist").numpy()
    assert abs(rho - spearmanr(t[iu], dd[iu])[0]) < 1e-4


def test_config5_generalisation_matches_oracle():
    """BASELINE configs[4], end to end (HiC_GAT_generalize_directly.py:101-336): KR-normalise both
    chr19 resolutions on the device, train the flagship on 1 mb with the COMBINED loss against
    cont2dist(y, 1) for K fixed steps, generalise to 500 kb (Procrustes on the device, load_input,
    get_model, dSCC vs cont2dist(y_500kb, 1)); tests/golden/make_config5_band.py ran the oracle on
    the same inputs at 1/2/4/8 threads and seeds 0..3.

    * teacher-forced: the ORACLE's trained weights (1 thread, seed 0) and its Procrustes fit through
      the device's load_input / get_model / dSCC must give the oracle's generalised dSCC (no
      training chaos: within 1e-3);
    * free-running: the device's own K-step training must reach the oracle's trained-resolution
      dSCC within +-0.005 of the 1-thread value (the oracle's own spread there is ~4e-3), and its
      generalised dSCC must fall inside the oracle's run-to-run band (+-0.02): extrapolating to
      another resolution turns rounding-level training differences into a 0.05-wide spread in the
      oracle itself (0.35-0.47 over threads / seeds), so +-0.005 against one oracle run is not a
      property the reference has there."""
    import hicgat
    band = load_golden("config5_band_chr19.npz")
    K = int(band["steps"])
    th, sd = band["threads"], band["seeds"]
    ref_i = int(np.flatnonzero((th == 1) & (sd == 0))[0])
    al = load_golden("align_chr19_f512.npz")
    scale = float(band["feature_scale"])
    e1 = (scale * al["emb1"]).astype(np.float32)
    e2 = (scale * al["emb2"]).astype(np.float32)
    normed = {}
    for tag in ("1mb", "500kb"):
        a = np.array(load_golden(f"graph_chr19_{tag}.npz")["matrix"], dtype=np.float64)
        np.fill_diagonal(a, 0)
        normed[tag] = hicgat.kr.KRnorm(a)[0].cpu().numpy()
    # teacher-forced generalisation of the oracle's trained model, on the oracle's (scipy) Procrustes
    # fit: with 512 columns and ~116 matched bins the rotation is not unique on the null space, so
    # the device's own fit (tested for the optimum by test_domain_alignment_device_rank_deficient_*)
    # may differ there
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    sdict = {k[2:]: torch.tensor(band[k]) for k in band if k.startswith("w:")}
    model.load_state_dict(sdict)
    d5 = hicgat.load_input(normed["500kb"].copy(), np.asarray(band["fit500"], dtype=np.float32))
    model.eval()
    with torch.no_grad():
        c5 = model.get_model(d5.x.float(), d5.edge_index)
    rho_tf = hicgat.metrics.dscc(c5, hicgat.cont2dist(d5.y, 1).float())
    g_ref = float(band["dscc_generalised"][ref_i])
    # free-running device training
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    data = hicgat.load_input(normed["1mb"], e1)
    truth = hicgat.Truth.from_contacts(data.y, 1)
    _, hist = hicgat.train.train(model, data, truth, steps=K, loss="combined")
    with torch.no_grad():
        coords = model.get_model(data.x.float(), data.edge_index)
    rho_tr = hicgat.metrics.dscc(coords, truth.scoring())
    rho_gen, _ = hicgat.align.generalize(model, al["list1"], al["list2"], e1, e2, normed["500kb"], 1)
    gb, tb = np.asarray(band["dscc_generalised"]), np.asarray(band["dscc_trained"])
    print(f"[config5] K={K} teacher-forced generalised dSCC: device {rho_tf:.6f} vs oracle {g_ref:.6f} "
          f"(|diff| {abs(rho_tf - g_ref):.1e}); free-running: trained 1mb dSCC device {rho_tr:.6f} vs oracle "
          f"1-thread {tb[ref_i]:.6f} (oracle runs {np.round(tb, 4)}), generalised 500kb dSCC device {rho_gen:.6f}, "
          f"oracle runs (threads {list(th)}, seeds {list(sd)}) {np.round(gb, 4)}; final loss device {hist[-1]:.6e} "
          f"vs oracle {float(band['loss'][ref_i]):.6e}")
    assert abs(rho_tf - g_ref) <= 1e-3, (rho_tf, g_ref)
    assert abs(rho_tr - float(tb[ref_i])) <= 0.005, (rho_tr, tb)
    # the generalised dSCC of ONE free run moves by ~0.04 under a rounding change (the oracle's own
    # seed 0 at 1/2/4/8 threads: 0.339-0.376): checked on the seed median, test below
    assert 0.0 < rho_gen < 1.0, rho_gen


def _config5_inputs():
    import hicgat
    band = load_golden("config5_band_chr19.npz")
    al = load_golden("align_chr19_f512.npz")
    scale = float(band["feature_scale"])
    e1 = (scale * al["emb1"]).astype(np.float32)
    e2 = (scale * al["emb2"]).astype(np.float32)
    normed = {}
    for tag in ("1mb", "500kb"):
        a = np.array(load_golden(f"graph_chr19_{tag}.npz")["matrix"], dtype=np.float64)
        np.fill_diagonal(a, 0)
        normed[tag] = hicgat.kr.KRnorm(a)[0].cpu().numpy()
    return al, e1, e2, normed


@pytest.mark.timeout(900)
def test_config5_generalisation_seed_median_matches_oracle():
    """BASELINE configs[4] free-running, on the seed protocol of the chr19 1 mb north-star check:
    train on 1 mb (combined loss, K = 1000, initial-weight seeds 0..23), generalise to 500 kb
    (HiC_GAT_generalize_directly.py:312-336); the MEDIAN generalised dSCC over the seeds within
    +-0.01 of the oracle's median over the same seeds at 1 thread (tests/golden/make_config5_seeds.py).
    The same fixture holds the oracle at 2 threads -- another fp32 summation order of the same
    arithmetic, i.e. what a rounding change alone does: its median sits 2.1e-3 from the 1-thread one,
    so +-0.01 is ~5x the rounding-level movement of the statistic, while one seed's value moves by up
    to 0.04 (seed 0: 0.346 / 0.380)."""
    import hicgat
    fx = load_golden("config5_seeds_chr19.npz")
    K = int(fx["steps"])
    one = fx["threads"] == 1
    seeds = [int(v) for v in fx["seeds"][one]]
    ref = np.asarray(fx["dscc_generalised"][one], dtype=np.float64)
    ref2 = np.asarray(fx["dscc_generalised"][fx["threads"] == 2], dtype=np.float64)
    al, e1, e2, normed = _config5_inputs()
    data = hicgat.load_input(normed["1mb"], e1)
    truth = hicgat.Truth.from_contacts(data.y, 1)
    dev = []
    for sd in seeds:
        torch.manual_seed(sd)
        model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
        hicgat.train.train(model, data, truth, steps=K, loss="combined")
        rho, _ = hicgat.align.generalize(model, al["list1"], al["list2"], e1, e2, normed["500kb"], 1)
        dev.append(rho)
    dev = np.asarray(dev)
    with np.printoptions(precision=4):
        print(f"[config5 seeds] K={K} generalised 500 kb dSCC, seeds {seeds[0]}..{seeds[-1]}: device median "
              f"{np.median(dev):.6f} (mean {dev.mean():.6f}); oracle 1 thread median {np.median(ref):.6f} (mean "
              f"{ref.mean():.6f}), 2 threads {np.median(ref2):.6f}; |diff of medians| "
              f"{abs(np.median(dev) - np.median(ref)):.2e}; device {dev}; oracle {ref}")
    assert abs(np.median(dev) - np.median(ref)) <= 0.01, (np.median(dev), np.median(ref))


# ---------------------------------------------------------------- north star: dSCC band
@pytest.mark.parametrize("feats", ["fixture", "node2vec"])
def test_dscc_chr19_1mb_k3000_matches_oracle(feats):
    """feats = "node2vec": BASELINE configs[0]'s 512-d node2vec features -- the embedding this repo's
    GPU node2vec made with the reference's parameters (tests/golden/make_n2v_chr19.py), fed to both
    the device pipeline and the oracle band (make_dscc_band.py --features n2v).  With them the
    flagship collapses to constant coordinates in the oracle (dSCC undefined), so that case checks
    that the device lands on the same degenerate fixed point (final loss within 1e-3).

    BASELINE north star: dSCC on GM12878 chr19 1 mb within +-0.005 of the reference.  The
    HiC-GNN_main.py pipeline (:92-139) on the device -- hicgat.kr KR normalisation, load_input,
    cont2dist(y, 0.5), the fixture's 512-d features (node2vec is absent), seed-0
    initial weights, a fixed K = 3000 steps (the threshold stop is chaotic), get_model,
    Spearman of the upper-triangle distances -- against the CPU oracle's 1-thread dSCC of the same
    pipeline (tests/golden/make_dscc_band.py, run in the build container: K = 3000 at 1/2/4/8 threads;
    their spread is the oracle's own noise floor, printed beside the difference).  K = 3000 is where
    the training has settled: at K = 200 and K = 1000 the oracle's thread-count spread is 2.8e-3 and
    3.8e-2, at K = 3000 it is 3.3e-3."""
    import hicgat
    from oracle import kr as okr
    band = load_golden("dscc_band_chr19_1mb.npz" if feats == "fixture" else "dscc_band_chr19_1mb_n2v.npz")
    K = int(band["steps"])
    ref1 = float(band["dscc"][list(band["threads"]).index(1)])
    floor = float(band["dscc"].max() - band["dscc"].min())
    g = load_golden("graph_chr19_1mb.npz")
    mfx = load_golden("model_GATNetSelectiveResidualsUpdated.npz" if feats == "fixture" else "n2v_chr19_1mb.npz")
    a = np.array(g["matrix"], dtype=np.float64)
    np.fill_diagonal(a, 0)
    _, keep = okr.krnorm(a.copy())
    x = np.asarray(mfx["x"], dtype=np.float32)
    x = x[np.asarray(keep)] if len(keep) != len(x) else x
    normed_d, keep_d = hicgat.kr.KRnorm(a.copy())
    assert np.array_equal(keep_d.cpu().numpy(), np.asarray(keep))
    data = hicgat.load_input(normed_d.cpu().numpy(), x)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    tr = hicgat.Truth.from_contacts(data.y, 0.5)
    _, hist = hicgat.train.train(model, data, tr, steps=K)
    with torch.no_grad():
        coords = model.get_model(data.x.float(), data.edge_index)
    rho = hicgat.metrics.dscc(coords, tr.scoring())
    if feats == "node2vec":
        # with these node2vec features the oracle itself collapses to (near-)constant coordinates
        # at 1/2/4/8 threads (final loss 8.5743e-2 at 1, 4 and 8 threads, dSCC undefined / 0.0035):
        # the device must reach the same degenerate fixed point -- same final loss, no rank signal
        loss1 = float(band["loss"][list(band["threads"]).index(1)])
        print(f"[node2vec] device loss {hist[-1]:.6e} dSCC {rho}; oracle 1 thread loss {loss1:.6e}, "
              f"dSCC 1/2/4/8 threads {band['dscc']}")
        assert abs(hist[-1] - loss1) <= 1e-3 * loss1, (hist[-1], loss1)
        assert not (abs(rho) > 0.05), rho
        return
    print(f"[{feats}] dSCC chr19 1mb after {K} steps: device {rho:.6f}; oracle 1 thread {ref1:.6f} "
          f"(|diff| {abs(rho - ref1):.2e}); oracle 1/2/4/8 threads {np.round(band['dscc'], 6)} "
          f"(noise floor {floor:.2e})")
    assert abs(rho - ref1) <= 0.005, (rho, ref1)


def _chr19_device_dscc(x_fix, seed, K):
    """The device HiC-GNN_main.py pipeline on chr19 1 mb (KR, load_input, cont2dist(y, 0.5), weights
    from ``seed``, K fixed steps, get_model, dSCC); returns (dSCC, the Adj used)."""
    import hicgat
    from oracle import kr as okr
    g = load_golden("graph_chr19_1mb.npz")
    a = np.array(g["matrix"], dtype=np.float64)
    np.fill_diagonal(a, 0)
    _, keep = okr.krnorm(a.copy())
    x = np.asarray(x_fix, dtype=np.float32)
    x = x[np.asarray(keep)] if len(keep) != len(x) else x
    normed_d, _ = hicgat.kr.KRnorm(a.copy())
    data = hicgat.load_input(normed_d.cpu().numpy(), x)
    torch.manual_seed(seed)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    tr = hicgat.Truth.from_contacts(data.y, 0.5)
    hicgat.train.train(model, data, tr, steps=K)
    with torch.no_grad():
        coords = model.get_model(data.x.float(), data.edge_index)
    return hicgat.metrics.dscc(coords, tr.scoring()), data.edge_index


@pytest.mark.parametrize("form", ["gather", "tiles"])
def test_dscc_chr19_1mb_seed_mean_matches_oracle_both_forms(form, monkeypatch):
    """The north-star dSCC check made robust to the summation order: the fixed-K endpoint of ONE
    run moves by about the oracle's own thread noise under any rounding change (one seed through the
    dense-tile aggregation lands 5.8e-3 from the oracle), and now and then a run
    settles in another basin (the oracle's own seed 2: 0.919 against 0.930-0.935 for the other
    seven; a device seed through the tiles: 0.87), so the protocol is the MEDIAN dSCC over
    initial-weight seeds 0..7 (K = 3000, the oracle at 1 thread: tests/golden/make_dscc_band.py
    --seeds).  Both device aggregation forms -- the wave-per-row gather (the product path for this
    graph) and the dense-tile MFMA form (forced on) -- must land within +-0.005 of the oracle's
    median; a mean over four seeds moved by 1.3e-2 with one device seed in another basin."""
    import hicgat
    band = load_golden("dscc_seeds_chr19_1mb.npz")
    K = int(band["steps"])
    seeds = [int(v) for v in band["seeds"]]
    ref = np.asarray(band["dscc"], dtype=np.float64)
    if form == "tiles":
        monkeypatch.setattr(hicgat.graph, "TILE_MIN_N", 0)
        monkeypatch.setattr(hicgat.graph, "TILE_FRAC", 0.0)
    x = load_golden("model_GATNetSelectiveResidualsUpdated.npz")["x"]
    dev = []
    for sd in seeds:
        rho, adj = _chr19_device_dscc(x, sd, K)
        assert (adj.tiles() is not None) == (form == "tiles")
        dev.append(rho)
    dev = np.asarray(dev)
    with np.printoptions(precision=6):
        print(f"[{form}] dSCC chr19 1mb K={K} seeds {seeds}: device {dev} median {np.median(dev):.6f} "
              f"mean {dev.mean():.6f}; oracle {ref} median {np.median(ref):.6f} mean {ref.mean():.6f}; "
              f"|diff of medians| {abs(np.median(dev) - np.median(ref)):.2e}; per-seed |diff| max "
              f"{np.abs(dev - ref).max():.2e}")
    assert abs(np.median(dev) - np.median(ref)) <= 0.005, (dev, ref)


@pytest.mark.parametrize("n", [1, 2, 3, 5])
def test_gatconv_tiny_graphs_match_oracle(n):
    """Degenerate inputs: a single node, nodes without any contact (rows = the self loop only),
    fewer rows than a wave / a block -- forward and backward against the oracle."""
    import hicgat
    a = np.zeros((n, n))
    if n >= 3:
        a[0, 2] = a[2, 0] = 4.0
    ref, mine = _gat_pair(seed=100 + n)
    adj = hicgat.Adj.from_dense_device(torch.tensor(a, device=DEV))
    rng = np.random.default_rng(n)
    x = torch.tensor((0.1 * rng.standard_normal((n, 512))).astype(np.float32))
    g = torch.tensor(rng.standard_normal((n, 512)).astype(np.float32))
    xr = x.clone().requires_grad_(True)
    out_r = ref(xr, (adj.storage.rowptr(), adj.storage.col()))
    (out_r * g).sum().backward()
    xm = x.to(DEV).requires_grad_(True)
    out_m = mine(xm, adj)
    (out_m * g.to(DEV)).sum().backward()
    np.testing.assert_allclose(out_m.detach().cpu().numpy(), out_r.detach().numpy(), rtol=1e-5, atol=1e-6)
    assert _rel(xm.grad.cpu(), xr.grad) < 1e-4
    for (name, pr), (_, pm) in zip(ref.named_parameters(), mine.named_parameters()):
        assert _rel(pm.grad.cpu(), pr.grad) < 1e-4 or pr.grad.abs().max() < 1e-30, name


# ---------------------------------------------------------------- a6: the tail's packed weight copies
def test_tail_pack_layout_and_bitwise_kernels():
    """hicgat_tail_pack: the forward (mfma_rows) and backward (mfma_rows_t) layouts of W1c / W2c / Wh
    against their index formulas, and the four one-kernel tail launches (plain and head-fused,
    forward and backward) reading the packed copies bitwise equal to the same launches reading the
    row-major weights (every lane holds the same values in the same registers).  M = 1030: a partial
    last workgroup."""
    from hicgat import kernels, ops
    K = kernels.default()
    torch.manual_seed(11)
    W1c, W2c, Wh = (torch.randn(n, n, device=DEV) * 0.05 for n in (512, 256, 512))
    pack = K.tail_pack(W1c, W2c, Wh).cpu()

    def fwd_layout(W):
        R, C = W.shape
        G = C // 32
        o = torch.arange(R * C // 4)
        L, chunk = o % 64, o // 64
        e, g, b = chunk % 2, (chunk // 2) % G, (chunk // 2) // G
        rows = 16 * b + L % 16
        cols = 32 * g + 8 * (L // 16) + 4 * e
        return torch.stack([W[rows, cols + c] for c in range(4)], 1).reshape(-1)

    def bwd_layout(W):
        R, C = W.shape
        o = torch.arange(R * C // 4)
        L, blk = o % 64, o // 64
        g, cb = blk // (C // 16), blk % (C // 16)
        rows = 16 * g + 4 * (L // 16)
        cols = 16 * cb + L % 16
        return torch.stack([W[rows + c, cols] for c in range(4)], 1).reshape(-1)

    Wc = [w.cpu() for w in (W1c, W2c, Wh)]
    want = torch.cat([fwd_layout(Wc[0]), fwd_layout(Wc[1]), fwd_layout(Wc[2]),
                      bwd_layout(Wc[0]), bwd_layout(Wc[1]), bwd_layout(Wc[2])])
    assert pack.shape == want.shape and torch.equal(pack, want)

    M = 1030
    f = dict(device=DEV)
    x = torch.relu(torch.randn(M, 512, **f))
    small = [torch.randn(n, **f) * 0.1 for n in (512, 256, 256, 256, 128, 128, 64, 64, 64)]
    b1c, g1, be1, b2c, g2, be2, b3, g3, be3 = small
    g1, g2, g3 = 1 + g1, 1 + g2, 1 + g3
    W3, W4, b4 = torch.randn(64, 128, **f) * 0.1, torch.randn(3, 64, **f) * 0.1, torch.randn(3, **f) * 0.1
    dc = torch.randn(M, 3, **f)
    X4 = torch.randn(2, 2, M, 512, **f)
    bias = torch.randn(512, **f) * 0.1
    rs_init = torch.randn(M, 8, **f)
    for heads in (False, True):
        outs = []
        for pk in (None, K.tail_pack(W1c, W2c, Wh if heads else None)):
            h = None
            xin = x.clone()
            if heads:
                h = ops.TailHeads(X4, Wh, bias, torch.empty(M, 512, **f), torch.empty(M, 512, **f),
                                  rs_init.clone(), torch.empty(M, 1024, **f), act=1)
            coords, saved = K.tail_fwd_fused(xin, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4, 1e-5,
                                             heads=h, pack=pk)
            rs0 = h.rs.clone() if heads else None
            dx, dY1, dY2, dy3, ws = K.tail_bwd_fused(dc, saved, W4, W3, W2c, W1c, g1, be1, g2, be2, g3, be3, heads=h,
                                                     pack=pk)
            torch.cuda.synchronize()
            o = [coords, *saved, dY1, dY2, dy3, *ws]
            if heads:
                o += [xin, h.Y0, h.dout, h.dxa, h.rs, rs0]
            else:
                o += [dx]
            outs.append([t.detach().cpu().clone() for t in o])
        for a, b in zip(*outs):
            assert torch.equal(a, b), (heads, a.shape)


# ---------------------------------------------------------------- a6: the fused MLP-tail forward
@pytest.mark.parametrize("m,sinks,bwd", [(2701, False, True), (2701, True, True), (2701, True, False),
                                         (16000, True, True), (1030, False, True)])
def test_fused_tail_matches_per_layer_path(monkeypatch, m, sinks, bwd):
    """GATNetSelectiveResidualsUpdated.post_act through the one-launch forward and backward
    (tail_fused.hip; bwd=False: the per-layer backward steps on the fused forward's tensors) vs the
    per-layer kernels: coords, the input gradient and every tail parameter's gradient (into
    FlatAdam's gradient sinks, or autograd's .grad), and an fp64 torch evaluation of the forward.
    Tolerances: coords 1e-5 of their max (fp32 GEMM order), gradients 1e-4 of each tensor's max."""
    import hicgat
    from hicgat import ops
    monkeypatch.setattr(ops, "FUSED_TAIL_BWD", bwd)
    torch.manual_seed(7)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    with torch.no_grad():      # trained-looking LayerNorm affine parameters (beta != 0 moves the kinks)
        for nm in ("norm_a", "norm1", "norm2"):
            getattr(model, nm).weight.add_(0.1 * torch.randn_like(getattr(model, nm).weight))
            getattr(model, nm).bias.add_(0.1 * torch.randn_like(getattr(model, nm).bias))
    x0 = torch.relu(torch.randn(m, 512, device=DEV))
    g = torch.randn(m, 3, device=DEV)
    # the tail is row-wise: rows holding a relu input within 1e-5 of the kink (where the two fp32 GEMM
    # orders may take different sides, tests/kinks.py) get no upstream gradient, so
    # neither path's backward sees them
    d = torch.float64

    def lin(layer, v):
        return v @ layer.weight.detach().to(d).t() + layer.bias.detach().to(d)

    def ln(norm, v):
        return torch.nn.functional.layer_norm(v, v.shape[1:], norm.weight.detach().to(d), norm.bias.detach().to(d),
                                              norm.eps)

    with torch.no_grad():
        v = x0.to(d)
        p1 = ln(model.norm_a, lin(model.densea, v))
        v = torch.relu(p1) + lin(model.align_densea, v)
        p2 = ln(model.norm1, lin(model.dense1, v))
        v = torch.relu(p2) + lin(model.align_dense1, v)
        p3 = ln(model.norm2, lin(model.dense2, v))
        ref = lin(model.dense3, torch.relu(p3))
        kink = torch.cat([p1, p2, p3], 1).abs().amin(1) < 1e-5
    g[kink] = 0.0
    assert kink.float().mean().item() < 0.02
    tail = [p for n, p in model.named_parameters() if not n.startswith("conv.")]
    res = {}
    monkeypatch.setattr(ops, "FUSED_TAIL_MAX_M", max(m, ops.FUSED_TAIL_MAX_M))   # the kernel at N = 20000 too
    for fused in (False, True):
        monkeypatch.setattr(ops, "FUSED_TAIL", fused)
        assert ops.fused_tail_ok(model, x0) == fused
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3) if sinks else None
        if opt is not None:
            opt.zero_grad()
        else:
            for p in model.parameters():
                p.grad = None
        x = x0.clone().requires_grad_(True)
        with ops.overlapped_param_grads(sinks):
            c = model.post_act(x)
            c.backward(g)
        torch.cuda.synchronize()
        res[fused] = (c.detach().clone(), x.grad.clone(), [p.grad.detach().clone() for p in tail])
    (c0, dx0, gp0), (c1, dx1, gp1) = res[False], res[True]
    assert _rel(c1.cpu(), c0.cpu()) < 1e-5
    assert (dx1 - dx0).abs().max().item() <= 1e-4 * dx0.abs().max().item()
    names = [n for n, _ in model.named_parameters() if not n.startswith("conv.")]
    for nm, a, b in zip(names, gp0, gp1):
        if nm == "dense3.bias":
            continue      # exactly 0 up to rounding when the upstream gradient sums to ~0
        assert (b - a).abs().max().item() <= 1e-4 * a.abs().max().item(), nm
    assert _rel(c1.double().cpu(), ref.cpu()) < 1e-5      # the fp64 forward of models.py:638-659


@pytest.mark.parametrize("n,graphed", [(3000, False), (3000, True), (20000, False)])
def test_rows_pass_fused_into_tail_backward_is_bitwise(monkeypatch, n, graphed):
    """The single-GPU GATConv's rows pass (dout = g relu'(y), delta, da_dst; hicgat_gat_agg_bwd_rows)
    run in the one-kernel tail backward's epilogue (hicgat_tail_bwd_fused_rows, ops.FUSE_ROWS) against
    the separate pass: two training steps (eager, or captured and replayed) give the same loss,
    gradients and parameters bit for bit (same arithmetic on the same dx values)."""
    import hicgat
    from hicgat import ops, synth
    i, j, c = synth.contact_pairs(n, density=0.05 if n < 20000 else 0.01, seed=3)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    del A
    x = torch.tensor(synth.features(n, seed=3), device=DEV)
    res = {}
    for fuse in (False, True):
        monkeypatch.setattr(ops, "FUSE_ROWS", fuse)
        torch.manual_seed(0)
        model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
        assert ops.fused_tail_ok(model, torch.empty(n, 512, device=DEV))
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
        out = []
        if graphed:
            step = hicgat.graphs.captured_train_step(model, opt, x, adj, tr, warmup=1)
            for _ in range(2):
                loss = float(step()[0])
                out.append((loss, opt.grad.clone(), opt.flat.clone()))
        else:
            for _ in range(2):
                loss, _, _ = hicgat.train.train_step(model, opt, x, adj, tr)
                out.append((float(loss), opt.grad.clone(), opt.flat.clone()))
        torch.cuda.synchronize()
        res[fuse] = out
    for (l0, g0, p0), (l1, g1, p1) in zip(res[False], res[True]):
        assert l0 == l1 and torch.equal(g0, g1) and torch.equal(p0, p1)


@pytest.mark.parametrize("n", [3000, 20000])
def test_step_pack_in_first_launch_is_bitwise(monkeypatch, n):
    """The one-kernel tail's packed weights written by the training step's first launch
    (hicgat_step_begin_pack via ops.step_pack / FlatAdam.zero_grad(pack=...)) against the forward's
    own hicgat_tail_pack launch: two training steps give the same loss, gradients and parameters bit
    for bit, and the step's buffer holds exactly the packed copy of the step's weights."""
    import hicgat
    from hicgat import kernels, ops, synth
    i, j, c = synth.contact_pairs(n, density=0.05 if n < 20000 else 0.01, seed=5)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    del A
    x = torch.tensor(synth.features(n, seed=5), device=DEV)
    res = {}
    real = ops.step_pack
    for fold in (False, True):
        monkeypatch.setattr(ops, "step_pack", real if fold else (lambda model, x: None))
        torch.manual_seed(0)
        model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
        out = []
        for _ in range(2):
            if fold:
                m = model
                W1c = torch.cat([m.densea.weight, m.align_densea.weight]).detach()
                W2c = torch.cat([m.dense1.weight, m.align_dense1.weight]).detach()
                want = kernels.default().tail_pack(W1c, W2c)
            loss, _, _ = hicgat.train.train_step(model, opt, x, adj, tr)
            if fold:
                torch.cuda.synchronize()
                # the F1, F2, B1 and B2 regions (the head regions FH, BH stay unwritten without Wh)
                fh, b1, bh = 512 * 512 + 256 * 256, 2 * 512 * 512 + 256 * 256, 3 * 512 * 512 + 2 * 256 * 256
                got = model._hicgat_pack_buf
                for r0, r1 in ((0, fh), (b1, bh)):
                    assert torch.equal(got[r0:r1], want[r0:r1]), (r0, r1)
            out.append((float(loss), opt.grad.clone(), opt.flat.clone()))
        torch.cuda.synchronize()
        res[fold] = out
    for (l0, g0, p0), (l1, g1, p1) in zip(res[False], res[True]):
        assert l0 == l1 and torch.equal(g0, g1) and torch.equal(p0, p1)


@pytest.mark.parametrize("M", [4097, 9001, 20000])
def test_persistent_tail_forward_is_bitwise_the_tile_grid(M):
    """More row tiles than CUs: the one-kernel tail forward runs as one workgroup per CU walking the
    tiles, the next tile's x rows copied into LDS by LDS-DMA during the current one (tail_fused.hip
    PERSIST).  Against the same launch on row slices of at most 4 096 rows (256 tiles: one tile per
    workgroup), every output -- coordinates and the nine saved tensors -- is bitwise the same, with
    and without the packed weights; M = 4097 / 9001: a partial last tile."""
    from hicgat import kernels
    K = kernels.default()
    torch.manual_seed(13)
    f = dict(device=DEV)
    W1c, W2c = torch.randn(512, 512, **f) * 0.05, torch.randn(256, 256, **f) * 0.05
    small = [torch.randn(n, **f) * 0.1 for n in (512, 256, 256, 256, 128, 128, 64, 64, 64)]
    b1c, g1, be1, b2c, g2, be2, b3, g3, be3 = small
    g1, g2, g3 = 1 + g1, 1 + g2, 1 + g3
    W3, W4, b4 = torch.randn(64, 128, **f) * 0.1, torch.randn(3, 64, **f) * 0.1, torch.randn(3, **f) * 0.1
    x = torch.relu(torch.randn(M, 512, **f))
    args = (W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4, 1e-5)
    for pk in (None, K.tail_pack(W1c, W2c)):
        coords, saved = K.tail_fwd_fused(x, *args, pack=pk)
        parts = [K.tail_fwd_fused(x[r0:r0 + 4096], *args, pack=pk) for r0 in range(0, M, 4096)]
        torch.cuda.synchronize()
        assert torch.equal(coords, torch.cat([c for c, _ in parts]))
        for k, t in enumerate(saved):
            assert torch.equal(t, torch.cat([s[k] for _, s in parts])), k
