"""GPU: the alternative fast kernels against the reference-form kernels on the same inputs.

* the x3 (three-way bf16 split) GEMM vs fp64 and the fp32-MFMA GEMM;
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
