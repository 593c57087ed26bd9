"""GPU: the alternative fast kernels against the reference-form kernels on the same inputs.

* the fp32-MFMA GEMM family vs fp64 (every layout / tile path), the fused linear + logits kernel;
* the split LayerNorm backward (parameter reduction on a second stream) vs the one-call form.
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


# ---------------------------------------------------------------- fp32 GEMM family (csrc/gemm.hip)
@pytest.mark.parametrize("a_km,b_km,m,n,k,splits", [
    (0, 0, 20000, 512, 512, 1),    # lin_l / Linear forward (the tall 160 x 128 kernel)
    (0, 0, 3001, 256, 512, 1),     # ragged M
    (0, 1, 5003, 512, 256, 1),     # input gradient
    (1, 1, 512, 512, 20000, 64),   # weight gradient, split K
    (1, 1, 256, 512, 4999, 7),     # ragged K and splits
    (0, 0, 130, 64, 20, 1),        # K not a multiple of the 16-deep K-step
])
def test_gemm_fp32_matches_fp64(a_km, b_km, m, n, k, splits):
    """Every layout / tile path of the fp32-MFMA GEMM against fp64, with the bias and accumulate
    epilogues (the GEMM tolerance of test_gpu_parity.py)."""
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(m + n + k)
    A = torch.randn((k, m) if a_km else (m, k), device=DEV)
    B = torch.randn((k, n) if b_km else (n, k), device=DEV)
    bias = None if a_km else torch.randn(n, device=DEV)
    ref = (A.double().t() if a_km else A.double()) @ (B.double() if b_km else B.double().t())
    if bias is not None:
        ref = ref + bias.double()
    tol = 5e-6 * max(1.0, (k / splits / 512) ** 0.5)
    C = torch.full((m, n), float("nan"), device=DEV)
    K.gemm(a_km, b_km, m, n, k, A, B, C, bias=bias, splits=splits)
    assert _rel(C.cpu(), ref.cpu()) < tol
    acc = torch.ones(m, n, device=DEV)
    K.gemm(a_km, b_km, m, n, k, A, B, acc, bias=bias, accumulate=True, splits=splits)
    assert _rel(acc.cpu(), (ref + 1).cpu()) < tol


def test_gemm_x3_arithmetic_is_refused():
    """HICGAT_GEMM_X3 was removed (measured slower per step): the ABI refuses it loudly."""
    import hicgat
    from hicgat import _lib
    K = hicgat.kernels.default()
    A = torch.randn(777, 64, device=DEV)
    W = torch.randn(64, 64, device=DEV)
    C = torch.empty(777, 64, device=DEV)
    with pytest.raises(_lib.HicgatError):
        K.gemm(0, 0, 777, 64, 64, A, W, C, impl=2)


def test_linear_att_fused_kernel_matches_gemm_path():
    """hicgat_gat_linear_att (the 64x256-tile GEMM with the logits in its epilogue) vs the product
    path (tall GEMM + logits pass) and fp64."""
    import hicgat
    from hicgat import _lib
    K = hicgat.kernels.default()
    torch.manual_seed(2)
    n = 4097
    x = torch.randn(n, 512, device=DEV) * 0.1
    W = torch.randn(512, 512, device=DEV) * 0.05
    al = torch.randn(1, 2, 256, device=DEV)
    ar = torch.randn(1, 2, 256, device=DEV)
    h1, s1, d1 = K.linear_att(x, W, al, ar)
    h2, s2, d2 = torch.empty_like(h1), torch.empty_like(s1), torch.empty_like(d1)
    P = _lib.ptr
    _lib.check(K.lib.hicgat_gat_linear_att(P(x), P(W), P(al), P(ar), n, 512, 2, 256, P(h2), P(s2), P(d2),
                                           _lib.stream(x.device)), "hicgat_gat_linear_att")
    href = x.double() @ W.double().t()
    hv = href.view(n, 2, 256)
    for h, s, d in ((h1, s1, d1), (h2, s2, d2)):
        assert _rel(h.cpu(), href.cpu()) < 5e-6
        assert _rel(s.cpu(), (hv * al.double()).sum(-1).cpu()) < 1e-5
        assert _rel(d.cpu(), (hv * ar.double()).sum(-1).cpu()) < 1e-5


@pytest.mark.parametrize("W", [64, 128, 256])
def test_ln_bwd_split_params_same_bits(W):
    """hicgat_ln_relu_res_bwd with dgamma = dbeta = NULL + hicgat_ln_relu_res_bwd_params on a
    second stream (the deferred side-work form) == the one-call backward, bit for bit."""
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


@pytest.mark.parametrize("b_km", [0, 1])
@pytest.mark.parametrize("splits", [None, 1, 3])
def test_gemm_rows_grouped_matches_fp64(b_km, splits):
    """hicgat_gemm_rows_grouped (the xagg step's per-head GEMMs and dxa GEMMs): two jobs of a rank's
    shard shape in one launch, K split into slabs (None: the auto split) or written directly
    (splits = 1), bias and the relu copy, against fp64."""
    import hicgat
    K = hicgat.kernels.default()
    torch.manual_seed(7 + b_km)
    M, Kd, N = 2701, 256 if b_km else 512, 512 if b_km else 256
    jobs, refs = [], []
    for hd in range(2):
        A = torch.randn(M, Kd, device=DEV)
        B = torch.randn((Kd, N) if b_km else (N, Kd), device=DEV)
        C = torch.full((M, N), float("nan"), device=DEV)
        bias = None if b_km else torch.randn(N, device=DEV)
        Cr = None if b_km else torch.full((M, N), float("nan"), device=DEV)
        ref = A.double() @ (B.double() if b_km else B.double().t())
        if bias is not None:
            ref = ref + bias.double()
        jobs.append((A, B, C, bias, Cr))
        refs.append(ref)
    K.gemm_rows_grouped(jobs, b_kmajor=b_km, splits=splits)
    for (A, B, C, bias, Cr), ref in zip(jobs, refs):
        assert _rel(C.cpu(), ref.cpu()) < 5e-6
        if Cr is not None:
            assert torch.equal(Cr, torch.relu(C))
