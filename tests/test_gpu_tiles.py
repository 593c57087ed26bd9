"""The dense-tile aggregation (csrc/gat_tiles.hip) against the gather kernels on the same inputs.

The tiled path computes the same GATConv training-form forward (a4+a5: out, out2, row stats) and
source-side backward (dh, da_src) as ``hicgat_gat_agg_fwd_act`` / ``hicgat_gat_agg_bwd_src_ld``,
with the edges of dense 32x32 tiles summed on the matrix cores in another order.  Graphs: ragged
sizes (a partial last row block and column block), a banded Hi-C-like graph, a fully dense one,
isolated rows (only the self loop), and tile thresholds from "every non-empty tile" (1) to "no tile"
(1025).  Tolerance: 1e-5 of each tensor's max (fp32 reassociation); the softmax statistics (max,
sum) come from the same gather pass and must be bitwise equal.  The fp64 check at synth-20000 is
tests/test_gpu_fullsize.py::test_synth20000_gat_backward_matches_fp64[tiled].
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
    import hicgat  # noqa: F401


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _graph(kind, n, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "dense":
        A = np.ones((n, n))
    elif kind == "band":   # Hi-C-like: |i-j|^-1 keep rate, first diagonals whole
        d = np.abs(np.arange(n)[:, None] - np.arange(n)[None, :])
        A = (rng.random((n, n)) < np.minimum(1.0, 6.0 / np.maximum(d, 1))).astype(float)
    elif kind == "random":
        A = (rng.random((n, n)) < 0.05).astype(float)
    elif kind == "isolated":   # a band graph with some loci contacting nothing
        d = np.abs(np.arange(n)[:, None] - np.arange(n)[None, :])
        A = (d <= 3).astype(float)
        iso = rng.choice(n, size=n // 10, replace=False)
        A[iso, :] = 0
        A[:, iso] = 0
    A = np.triu(A, 1)
    A = A + A.T
    import hicgat
    return hicgat.Adj.from_dense_device(torch.tensor(A, dtype=torch.float64, device=DEV), keep_host=False)


def _run(K, adj, n, tiles, seed=1):
    torch.manual_seed(seed)
    h = 0.5 * torch.randn(n, 512, device=DEV)
    att_l = 0.1 * torch.randn(1, 2, 256, device=DEV)
    att_r = 0.1 * torch.randn(1, 2, 256, device=DEV)
    bias = 0.05 * torch.randn(512, device=DEV)
    a_s, a_d = K.att_logits(h, att_l, att_r)
    out = torch.empty(n, 512, device=DEV)
    out2 = torch.empty(n, 512, device=DEV)
    rs = torch.empty(n, 8, device=DEV)
    if tiles is None:
        K.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, bias, 0.2, 1, out, out2, rs)
    else:
        K.agg_fwd_tiled(adj.rowptr32, adj.col32, tiles, h, a_s, a_d, bias, 0.2, 1, out, out2, rs)
    g = torch.randn(n, 512, device=DEV)
    dout = torch.empty(n, 512, device=DEV)
    K.agg_bwd_rows(0, n, 1, g, out, bias, out2, dout, rs)
    dh = torch.empty(n, 512, device=DEV)
    da_src = torch.empty(n, 2, device=DEV)
    if tiles is None:
        K.agg_bwd_src(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, rs, dout, att_l, att_r, 0.2, dh, da_src)
    else:
        K.agg_bwd_src_tiled(tiles, h, a_s, a_d, rs, dout, att_l, att_r, 0.2, dh, da_src)
    torch.cuda.synchronize()
    return dict(out=out, out2=out2, rs=rs, dout=dout, dh=dh, da_src=da_src)


CASES = [("band", 100, 1, 1), ("band", 100, 64, 2), ("band", 1000, 64, 1), ("band", 1000, 64, 5),
         ("band", 1000, 1025, 1), ("dense", 67, 64, 1), ("dense", 300, 64, 1), ("dense", 300, 64, 4),
         ("dense", 2000, 64, 8), ("random", 515, 1, 1), ("random", 515, 64, 3), ("isolated", 200, 4, 1),
         ("isolated", 200, 4, 16)]


@pytest.mark.parametrize("kind,n,tmin,splits", CASES, ids=[f"{k}-{n}-t{t}-s{s}" for k, n, t, s in CASES])
def test_tiled_matches_gather(kind, n, tmin, splits):
    """splits > 1: a row block's tiles spread over several workgroups, partials added by the
    epilogue passes (more splits than a block has tiles leaves some workgroups with none)."""
    import hicgat
    K = hicgat.kernels.default()
    adj = _graph(kind, n)
    tiles = hicgat.graph.build_tiles(adj.rowptr32, adj.col32, 0, n, n, tmin)
    tiles.splits = splits
    if tmin > 1024:
        assert tiles.ntiles == 0
    else:
        assert tiles.ntiles > 0
    ref = _run(K, adj, n, None)
    got = _run(K, adj, n, tiles)
    assert torch.equal(got["rs"][:, :4], ref["rs"][:, :4])          # max, sum: same pass
    errs = {k: _rel(got[k], ref[k]) for k in ("out", "out2", "dout", "dh", "da_src")}
    errs["delta"] = _rel(got["rs"][:, 4:6], ref["rs"][:, 4:6])
    errs["da_dst"] = _rel(got["rs"][:, 6:8], ref["rs"][:, 6:8])
    print(kind, n, tmin, splits, f"tiles {tiles.ntiles} dense edges {tiles.n_dense}/{adj.device_nnz}",
          {k: f"{v:.1e}" for k, v in errs.items()})
    for k, v in errs.items():
        assert v < 1e-5, (k, errs)


def test_tiled_gat_conv_autograd_matches_gather(monkeypatch):
    """The module path (gat_conv -> Adj.tiles()) with tiling on vs off: forward values and every
    parameter gradient."""
    import hicgat
    n = 700
    adj = _graph("band", n, seed=3)
    x = 0.1 * torch.randn(n, 512, device=DEV)
    res = {}
    for tmin in (0, 32):
        monkeypatch.setattr(hicgat.graph, "TILE_MIN", tmin)
        monkeypatch.setattr(hicgat.graph, "TILE_FRAC", 0.0)
        torch.manual_seed(0)
        conv = hicgat.GATConv(512, 256, heads=2).to(DEV)
        y = conv(x, adj, act="relu")
        (y * torch.linspace(-1, 1, 512, device=DEV)).sum().backward()
        res[tmin] = (y.detach(), {k: p.grad.detach().clone() for k, p in conv.named_parameters()})
    assert adj.tiles(32) is not None and adj.tiles(0) is None
    res_tiled_used = adj._tiles[1] is not None
    assert res_tiled_used
    assert _rel(res[32][0], res[0][0]) < 1e-5
    for k in res[0][1]:
        assert _rel(res[32][1][k], res[0][1][k]) < 1e-4, k


def test_tiled_abi_rejects_bad_arguments():
    import hicgat
    from hicgat import _lib
    lib = _lib.lib()
    z = torch.zeros(16, device=DEV)
    p = _lib.ptr(z)
    s = _lib.stream()
    fwd = lambda nt, N, H, r0, r1, sp=1, ws=None, wb=0: lib.hicgat_gat_agg_fwd_tiled(  # noqa: E731
        p, p, p, p, p, p, p, nt, N, H, 256, r0, r1, p, p, p, p, 0.2, 1, p, p, p, sp, ws, wb, s)
    # negative ntiles, row range outside N, unsupported heads
    assert fwd(-1, 4, 2, 0, 4) != 0
    assert fwd(0, 4, 2, 0, 5) != 0
    assert fwd(0, 4, 1, 0, 4) != 0
    assert lib.hicgat_gat_agg_bwd_src_tiled(p, p, p, None, None, 3, 4, 2, 256, 0, 4, p, p, p, p, 8, p, 512, p, p,
                                            0.2, p, p, 1, None, 0, s) != 0
    # splits > 1 without (or with too small) a workspace; splits out of range
    need = lib.hicgat_gat_tiled_workspace_bytes(4, 2)
    assert need > 0 and lib.hicgat_gat_tiled_workspace_bytes(4, 1) == 0
    assert fwd(0, 4, 2, 0, 4, 2) != 0
    assert fwd(0, 4, 2, 0, 4, 2, p, need - 4) != 0
    assert fwd(0, 4, 2, 0, 4, 0) != 0 and fwd(0, 4, 2, 0, 4, 65) != 0
    # an empty range is a no-op
    assert fwd(0, 4, 2, 2, 2) == 0


def test_tile_policy_dense_vs_power_law(monkeypatch):
    """Adj.tiles(): the tiled form for a (nearly) dense contact map, the gather alone for a
    power-law graph whose dense tiles hold only part of the edges (HICGAT_TILE_FRAC)."""
    import hicgat
    from hicgat import synth
    dense = _graph("dense", 600)
    assert dense.tiles() is not None and dense.tiles().n_dense == dense.device_nnz
    assert _graph("dense", 100).tiles() is None          # a few row blocks: the gather alone
    n = 3000
    i, j, c = synth.contact_pairs(n, density=0.01, seed=0)
    sparse = hicgat.Adj.from_dense_device(synth.dense_contacts(n, i, j, c, device=DEV), keep_host=False)
    assert sparse.tiles() is None
    monkeypatch.setattr(hicgat.graph, "TILE_FRAC", 0.0)
    sparse._tiles = None
    assert sparse.tiles() is not None
