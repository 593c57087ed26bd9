"""GPU: the alternative fast kernels against the reference-form kernels on the same inputs.

* XCD column-strip GAT aggregation (csrc/gat_sliced.hip) vs the row-per-wave kernels
  (gat_fwd.hip / gat_bwd.hip), which tests/test_gpu_parity.py pins to the oracle.
Tolerances as in test_gpu_parity.py (max-abs error relative to the tensor's max magnitude).
"""
import numpy as np
import pytest
import torch

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


@pytest.mark.parametrize("sw", [32, 64])
@pytest.mark.parametrize("n,density", [(3000, 0.03), (20000, 0.01)])
def test_sliced_aggregation_matches_row_kernels(sw, n, density):
    """Row max / sum bit-identical, S3 to rounding; out, out2, dh, da_src to fp32 summation
    order; a row range (a rank's shard) writes only its rows."""
    import hicgat
    from hicgat import kernels, synth
    i, j, c = synth.contact_pairs(n, density=density, seed=11)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    A[5, :] = 0
    A[:, 5] = 0                                  # isolated row: self loop only
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    del A
    torch.manual_seed(4)
    h = torch.randn(n, 512, device=DEV) * 0.1
    a_s = torch.randn(n, 2, device=DEV)
    a_d = torch.randn(n, 2, device=DEV)
    b = torch.randn(512, device=DEV) * 0.1
    al = torch.randn(1, 2, 256, device=DEV)
    ar = torch.randn(1, 2, 256, device=DEV)
    row, sl = kernels.HipKernels(), kernels.HipKernels()
    row.slice_width, sl.slice_width = 0, sw
    res = []
    for K in (row, sl):
        out = torch.zeros(n, 512, device=DEV)
        out2 = torch.zeros_like(out)
        rs = torch.zeros(n, 8, device=DEV)
        K.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, 1, out, out2, rs)
        res.append((out, out2, rs))
    (o1, q1, rs1), (o2, q2, rs2) = res
    assert torch.equal(rs1[:, :4], rs2[:, :4])
    assert _rel(rs2[:, 4:6].cpu(), rs1[:, 4:6].cpu()) < 1e-6
    assert _rel(o2.cpu(), o1.cpu()) < 1e-5 and _rel(q2.cpu(), q1.cpu()) < 1e-5
    o3 = torch.zeros_like(o1)
    sl.agg_fwd(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, o3, torch.zeros_like(rs1))
    assert torch.equal(torch.relu(o3), o2)       # inference form = training form before the relu
    g = torch.randn(n, 512, device=DEV)
    dout = torch.empty_like(g)
    row.agg_bwd_rows(0, n, 1, g, o1, b, q1, dout, rs1)
    for r0, r1 in ((0, n), (n // 3, 2 * n // 3 + 1)):
        got = []
        for K in (row, sl):
            dh = torch.zeros(n, 512, device=DEV)
            da = torch.zeros(n, 2, device=DEV)
            K.agg_bwd_src(adj.rowptr32, adj.col32, r0, r1, h, a_s, a_d, rs1, dout, al, ar, 0.2, dh, da)
            got.append((dh, da))
        (dh1, da1), (dh2, da2) = got
        assert _rel(dh2[r0:r1].cpu(), dh1[r0:r1].cpu()) < 2e-5
        assert _rel(da2[r0:r1].cpu(), da1[r0:r1].cpu()) < 2e-5
        assert dh2[:r0].abs().sum().item() == 0 and dh2[r1:].abs().sum().item() == 0


def test_sliced_aggregation_strided_pack_and_long_rows():
    """The source pass reading dout / row stats from one packed [dout | stats] buffer (the
    multi-GPU layout) and rows of 2002 neighbours (many 64-record chunks, a ragged last one)."""
    import hicgat
    from hicgat import kernels
    n = 2003
    a = torch.ones(n, n, dtype=torch.float64, device=DEV)
    a.fill_diagonal_(0)
    adj = hicgat.Adj.from_dense_device(a, keep_host=False)
    torch.manual_seed(5)
    h = torch.randn(n, 512, device=DEV) * 0.1
    a_s = torch.randn(n, 2, device=DEV) * 3
    a_d = torch.randn(n, 2, device=DEV) * 3
    b = torch.zeros(512, device=DEV)
    al = torch.randn(1, 2, 256, device=DEV)
    ar = torch.randn(1, 2, 256, device=DEV)
    row, sl = kernels.HipKernels(), kernels.HipKernels()
    row.slice_width, sl.slice_width = 0, 32
    out = torch.empty(n, 512, device=DEV)
    out2 = torch.empty_like(out)
    rs = torch.empty(n, 8, device=DEV)
    row.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, 0, out, out2, rs)
    o_s = torch.empty_like(out)
    q_s = torch.empty_like(out)
    rs_s = torch.empty_like(rs)
    sl.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, 0, o_s, q_s, rs_s)
    assert _rel(o_s.cpu(), out.cpu()) < 1e-5 and _rel(q_s.cpu(), out2.cpu()) < 1e-5
    pack = torch.zeros(n, 512 + 8, device=DEV)
    g = torch.randn(n, 512, device=DEV)
    row.agg_bwd_rows(0, n, 0, g, out, b, out2, None, rs)
    pack[:, :512] = g
    pack[:, 512:] = rs
    res = []
    for K in (row, sl):
        dh = torch.empty(n, 512, device=DEV)
        da = torch.empty(n, 2, device=DEV)
        K.agg_bwd_src(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, pack[:, 512:], pack[:, :512], al, ar, 0.2, dh, da)
        res.append((dh.cpu(), da.cpu()))
    assert _rel(res[1][0], res[0][0]) < 2e-5 and _rel(res[1][1], res[0][1]) < 2e-5
    assert np.isfinite(res[1][0].numpy()).all()


# ---------------------------------------------------------------- x3 GEMM (csrc/gemm.hip)
@pytest.mark.parametrize("a_km,b_km,m,n,k,splits", [
    (0, 0, 20000, 512, 512, 1),    # lin_l / Linear forward
    (0, 0, 3001, 256, 512, 1),     # ragged M
    (0, 1, 5003, 512, 256, 1),     # input gradient
    (1, 1, 512, 512, 20000, 64),   # weight gradient, split K
    (1, 1, 256, 512, 4999, 7),     # ragged K and splits
    (0, 0, 130, 64, 20, 1),        # K not a multiple of the 16-deep K-step
])
def test_gemm_x3_is_as_accurate_as_fp32(a_km, b_km, m, n, k, splits):
    """The three-way bf16 split GEMM against fp64: error at most ~1.5x that of the fp32-MFMA kernel
    (which the reference's fp32 sgemm matches in class) and below the GEMM tolerance of
    test_gpu_parity.py; bias / accumulate epilogues identical in form."""
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(m + n + k)
    A = torch.randn((k, m) if a_km else (m, k), device=DEV)
    B = torch.randn((k, n) if b_km else (n, k), device=DEV)
    bias = None if a_km else torch.randn(n, device=DEV)
    ref = (A.double().t() if a_km else A.double()) @ (B.double() if b_km else B.double().t())
    if bias is not None:
        ref = ref + bias.double()
    err = {}
    for impl in (1, 2):
        C = torch.full((m, n), float("nan"), device=DEV)
        K.gemm(a_km, b_km, m, n, k, A, B, C, bias=bias, splits=splits, impl=impl)
        err[impl] = _rel(C.cpu(), ref.cpu())
    assert err[2] <= 1.5 * err[1] + 1e-7, err
    assert err[2] < 5e-6 * max(1.0, (k / splits / 512) ** 0.5), err
    acc = torch.ones(m, n, device=DEV)
    K.gemm(a_km, b_km, m, n, k, A, B, acc, bias=bias, accumulate=True, splits=splits, impl=2)
    assert _rel(acc.cpu(), (ref + 1).cpu()) < 5e-6 * max(1.0, (k / splits / 512) ** 0.5)


def test_gemm_x3_unsupported_shapes_fall_back():
    """N < 64 (dense3) or unaligned rows: impl x3 refuses (HICGAT_EUNSUPPORTED), auto runs fp32."""
    import hicgat
    from hicgat import _lib
    K = hicgat.kernels.default()
    A = torch.randn(777, 64, device=DEV)
    W = torch.randn(3, 64, device=DEV)
    C = torch.empty(777, 3, device=DEV)
    with pytest.raises(_lib.HicgatError):
        K.gemm(0, 0, 777, 3, 64, A, W, C, impl=2)
    K.gemm(0, 0, 777, 3, 64, A, W, C, impl=0)
    assert _rel(C.cpu(), (A.double() @ W.double().t()).cpu()) < 5e-6


def test_linear_att_x3_matches_fused_fp32_kernel():
    """The GATConv lin_l + logits as x3 GEMM + logits pass vs the fused fp32-MFMA kernel."""
    import hicgat
    from hicgat import kernels
    torch.manual_seed(2)
    n = 4097
    x = torch.randn(n, 512, device=DEV) * 0.1
    W = torch.randn(512, 512, device=DEV) * 0.05
    al = torch.randn(1, 2, 256, device=DEV)
    ar = torch.randn(1, 2, 256, device=DEV)
    f32, x3 = kernels.HipKernels(), kernels.HipKernels()
    f32.gemm_impl, x3.gemm_impl = 1, 2
    h1, s1, d1 = f32.linear_att(x, W, al, ar)
    h2, s2, d2 = x3.linear_att(x, W, al, ar)
    href = x.double() @ W.double().t()
    assert _rel(h2.cpu(), href.cpu()) <= 1.5 * _rel(h1.cpu(), href.cpu()) + 1e-7
    hv = href.view(n, 2, 256)
    assert _rel(s2.cpu(), (hv * al.double()).sum(-1).cpu()) < 1e-5
    assert _rel(d2.cpu(), (hv * ar.double()).sum(-1).cpu()) < 1e-5
    assert hicgat  # silence


@pytest.mark.parametrize("W", [64, 128, 256])
def test_ln_bwd_split_params_same_bits(W):
    """hicgat_ln_relu_res_bwd with dgamma = dbeta = NULL + hicgat_ln_relu_res_bwd_params on a
    second stream (the HICGAT_LN_SIDE form) == the one-call backward, bit for bit."""
    from hicgat import kernels
    K = kernels.default()
    M = 3001
    g = torch.Generator().manual_seed(W)
    y = torch.randn(M, W, generator=g).to(DEV)
    dz = torch.randn(M, W, generator=g).to(DEV)
    gamma = (1 + 0.1 * torch.randn(W, generator=g)).to(DEV)
    beta = (0.1 * torch.randn(W, generator=g)).to(DEV)
    z = torch.empty_like(y)
    stats = torch.empty(M, 2, device=DEV)
    K.ln_relu_res_fwd(y, gamma, beta, 1e-5, None, z, stats)
    dy1, dg1, db1 = torch.empty_like(y), torch.full((W,), 0.5, device=DEV), torch.full((W,), -0.5, device=DEV)
    K.ln_relu_res_bwd(dz, y, stats, gamma, beta, dy1, dg1, db1, accumulate=True)
    dy2, dg2, db2 = torch.empty_like(y), torch.full((W,), 0.5, device=DEV), torch.full((W,), -0.5, device=DEV)
    ws = K.ln_workspace(W, y.device)
    K.ln_relu_res_bwd(dz, y, stats, gamma, beta, dy2, None, None, ws=ws)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        K.ln_relu_res_bwd_params(W, dg2, db2, ws, accumulate=True)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(dy1, dy2) and torch.equal(dg1, dg2) and torch.equal(db1, db2)
