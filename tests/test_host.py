"""CPU: the C-ABI library loads and exports every symbol of include/hicgat.h (no compute calls),
and the host-side logic (list -> matrix, PDB writer, synthetic generator, tile counts)."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import GOLDEN, ROOT, load_golden


def _header_symbols():
    with open(os.path.join(ROOT, "include", "hicgat.h")) as fh:
        text = fh.read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(hicgat_\w+)\s*\(", text, re.M)))


def test_library_exports_every_header_symbol():
    from hicgat import _lib
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(syms)
    assert lib.hicgat_version() == 1
    assert b"unsupported" in lib.hicgat_strerror(-3)


def _header_arity():
    """{symbol: number of parameters} of every prototype in include/hicgat.h (comments stripped)."""
    with open(os.path.join(ROOT, "include", "hicgat.h")) as fh:
        text = re.sub(r"/\*.*?\*/", "", fh.read(), flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    out = {}
    for m in re.finditer(r"\b(hicgat_\w+)\s*\(([^;{]*?)\)\s*;", text, re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_ctypes_signatures_match_header_arity():
    """Every ctypes signature has as many arguments as the header's prototype (a miscounted
    signature fails only at call time, on a GPU)."""
    from hicgat import _lib
    arity = _header_arity()
    assert len(arity) >= 20
    for name, (_, args) in _lib.SIGNATURES.items():
        assert name in arity, name
        assert len(args) == arity[name], (name, len(args), arity[name])


def test_row_split_policy():
    """kernels.row_splits: the single-GPU N = 20000 GEMM shapes are never K-split; a rank's shard
    (N = 20000 over P = 2..8) is split only as far as ~512 workgroups and never below 128-deep
    K chunks."""
    from hicgat import kernels as hk
    dims = (3, 64, 128, 256, 512, 1024)
    for n_out in dims:
        for k in dims:
            assert hk.row_splits(20000, n_out, k) == 1
            assert hk.row_splits(20000, k, n_out) == 1
    for p in range(2, 9):
        m = -(-20000 // p)
        for n_out in (64, 128, 256, 512):
            for k in (256, 512, 1024):
                s = hk.row_splits(m, n_out, k)
                wgs = -(-m // 64) * -(-n_out // (128 if n_out >= 128 else 64))
                assert 1 <= s <= k // 128
                if s > 1:
                    assert wgs < 256 and wgs * (s - 1) < 512
    assert hk.row_splits(2500, 512, 128) == 1 and hk.row_splits(512, 512, 512) == 1


def test_query_functions_need_no_gpu():
    from hicgat import _lib
    lib = _lib.load()
    assert lib.hicgat_pairdist_num_tiles(20000, 1) == 157 * 158 // 2  # HICGAT_PD_TRI
    assert lib.hicgat_pairdist_num_tiles(20000, 0) == 157 * 157  # HICGAT_PD_SQUARE
    assert lib.hicgat_pairdist_num_tiles(0, 0) == 0
    assert lib.hicgat_pairdist_workspace_bytes(58, 1) > 0


def test_ops_fail_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import hicgat
    with pytest.raises(hicgat._lib.HicgatUnavailable):
        hicgat.ops.pairwise_dist(torch.zeros(4, 3))


@pytest.mark.parametrize("case", ["chr19_1mb", "chr19_500kb", "synth256"])
def test_convert_to_matrix_bit_exact(case):
    import hicgat
    g = load_golden(f"graph_{case}.npz")
    assert np.array_equal(hicgat.convert_to_matrix(g["list"]), g["matrix"])


def test_adj_host_surface_matches_reference_csr():
    import hicgat
    g = load_golden("graph_chr19_500kb.npz")
    a = g["matrix"].copy()
    np.fill_diagonal(a, 0)
    iu = np.argwhere(np.triu(a != 0, 1))
    adj = hicgat.Adj(torch.tensor(iu[:, 0]), torch.tensor(iu[:, 1]), torch.ones(len(iu)), (a.shape[0], a.shape[0]))
    sym = adj.to_symmetric()
    assert np.array_equal(sym.storage.rowptr().numpy(), g["rowptr"])
    assert np.array_equal(sym.storage.col().numpy(), g["col"])


@pytest.mark.parametrize("pdb", ["GM12878_1mb_chr19_list_structure.pdb",
                                 "GM12878_500kb_chr19_list_generalized_structure.pdb"])
def test_write_pdb_byte_exact_with_reference_output(tmp_path, pdb):
    from hicgat import io
    src = os.path.join(GOLDEN, pdb)
    xyz = io.read_pdb_coords(src)
    out = tmp_path / "o.pdb"
    io.write_pdb(xyz, str(out))
    assert out.read_bytes() == open(src, "rb").read()


def test_synthetic_generator_density_and_determinism():
    from hicgat import synth
    i, j, c = synth.contact_pairs(3000, density=0.01, seed=0)
    i2, j2, c2 = synth.contact_pairs(3000, density=0.01, seed=0)
    assert np.array_equal(i, i2) and np.array_equal(j, j2) and np.array_equal(c, c2)
    dens = 2 * len(i) / (3000 * 2999)
    assert abs(dens - 0.01) < 5e-4
    assert np.all(i < j) and np.all(c >= 1)
    i, j, c = synth.contact_pairs(200, density=None, seed=0)
    assert len(i) == 200 * 199 // 2


def test_adj_host_sage_weights_match_oracle():
    """Adj(row, col, value).to(device) derives the SAGEConv weights of the set_diag'd CSR and the
    1/degree normaliser on the host (no GPU needed for device='cpu')."""
    import hicgat
    from conftest import load_golden
    from oracle import sage
    g = load_golden("graph_chr19_500kb.npz")
    rp, c, v = (torch.tensor(g[k]) for k in ("rowptr", "col", "value"))
    n = rp.numel() - 1
    r = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
    adj = hicgat.Adj(r, c, v, (n, n)).to("cpu")
    rp2 = adj.rowptr32.long()
    c2 = adj.col32.long()
    r2 = torch.repeat_interleave(torch.arange(n), rp2[1:] - rp2[:-1])
    diag = r2 == c2
    assert diag.sum().item() == n and torch.all(adj.value32[diag] == 0)
    assert torch.equal(adj.value32[~diag], v.float())
    assert np.array_equal(adj.inv_deg.numpy(), sage.degree_inverse(g["rowptr"], g["col"], g["value"], n))


def test_adjacent_requires_one_storage():
    """ops._adjacent / _joined: views into one flat buffer join without a copy; two storages that
    merely sit back to back in memory (the caching allocator packs small blocks) do not."""
    import numpy as np
    from hicgat.ops import _adjacent, _joined
    flat = torch.arange(16, dtype=torch.float32)
    a, b = flat[:8].view(2, 4), flat[8:].view(2, 4)
    assert _adjacent(a, b)
    j = _joined(a, b)
    assert j.data_ptr() == a.data_ptr() and torch.equal(j, flat.view(4, 4))
    arr = np.arange(16, dtype=np.float32)
    x, y = torch.from_numpy(arr[:8]).view(2, 4), torch.from_numpy(arr[8:]).view(2, 4)
    assert y.data_ptr() == x.data_ptr() + 32 and x.untyped_storage().data_ptr() != y.untyped_storage().data_ptr()
    assert not _adjacent(x, y)
    assert torch.equal(_joined(x, y), torch.from_numpy(arr).view(4, 4))


@pytest.mark.parametrize("r0,r1,tmin", [(0, 150, 1), (0, 150, 20), (0, 150, 2000), (37, 121, 8)])
def test_build_tiles_partitions_the_edges(r0, r1, tmin):
    """hicgat.graph.build_tiles: every edge of rows [r0, r1) is in exactly one of a dense tile (bit
    set in its row's mask word) or the remainder CSR (order kept); every tile holds >= tmin edges
    and every tile that does is listed; rows outside the range are empty in the remainder."""
    from hicgat.graph import build_tiles
    rng = np.random.default_rng(5)
    n = 150
    d = np.abs(np.arange(n)[:, None] - np.arange(n)[None, :])
    A = (rng.random((n, n)) < np.minimum(1.0, 5.0 / np.maximum(d, 1))) | (d == 0)
    A = np.triu(A) | np.triu(A).T
    rowptr = np.zeros(n + 1, dtype=np.int32)
    rowptr[1:] = np.cumsum(A.sum(1))
    col = np.nonzero(A)[1].astype(np.int32)
    t = build_tiles(torch.tensor(rowptr), torch.tensor(col), r0, r1, n, tmin)
    tptr = t.tptr.numpy()
    tcol = t.tcol.numpy()
    mask = t.tmask.numpy().view(np.uint32)
    got = np.zeros((n, n), dtype=int)
    for b in range(len(tptr) - 1):
        for k in range(tptr[b], tptr[b + 1]):
            cnt = 0
            for i in range(32):
                for c in range(32):
                    if (int(mask[32 * k + i]) >> c) & 1:
                        got[r0 + 32 * b + i, 32 * tcol[k] + c] += 1
                        cnt += 1
            assert cnt >= tmin
    rps, cs = t.rowptr_s.numpy(), t.col_s.numpy()
    for r in range(n):
        seg = cs[rps[r]:rps[r + 1]]
        if not (r0 <= r < r1):
            assert len(seg) == 0
        assert np.all(np.diff(seg) > 0)
        got[r, seg] += 1
    want = np.zeros((n, n), dtype=int)
    want[r0:r1] = A[r0:r1]
    assert np.array_equal(got, want)
    assert t.n_dense == int(sum(bin(int(w)).count("1") for w in mask))
    # completeness: no tile left out that holds >= tmin edges
    for b in range((r1 - r0 + 31) // 32):
        rows = slice(r0 + 32 * b, min(r1, r0 + 32 * b + 32))
        for cb in range((n + 31) // 32):
            listed = cb in set(tcol[tptr[b]:tptr[b + 1]])
            assert listed == (A[rows, 32 * cb:32 * cb + 32].sum() >= max(tmin, 1))


def test_asymmetric_truth_scores_the_raw_upper_triangle():
    """an asymmetric target (R's KR rounding, r_utils.R:74-89) is stored symmetrised for
    the fused loss, but dSCC ranks the upper triangle AS GIVEN (HiC-GNN_main.py:135-139)."""
    import hicgat
    from scipy.stats import spearmanr
    rng = np.random.default_rng(5)
    n = 40
    t = rng.random((n, n))
    t = t + t.T
    t[np.triu_indices(n, 1)] *= 1 + 1e-3 * rng.standard_normal(n * (n - 1) // 2)   # rounding-size asymmetry
    np.fill_diagonal(t, 0)
    truth = hicgat.Truth(torch.tensor(t, dtype=torch.float32))
    assert truth.asymmetric_source
    d = truth.dense()
    assert torch.equal(d, d.t())
    iu = np.triu_indices(n, 1)
    raw = truth.scoring().numpy()
    assert np.array_equal(raw[iu], t.astype(np.float32)[iu])
    c = rng.standard_normal((n, 3))
    dist = np.linalg.norm(c[:, None] - c[None], axis=-1)[iu]
    rho_raw = spearmanr(raw[iu], dist)[0]
    assert rho_raw == spearmanr(t.astype(np.float32)[iu], dist)[0]
    sym = hicgat.Truth(torch.tensor(t + t.T, dtype=torch.float32))
    assert not sym.asymmetric_source and sym.scoring() is not None and torch.equal(sym.scoring(), sym.dense())
