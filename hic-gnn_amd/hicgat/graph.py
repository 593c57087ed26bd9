"""Graph and target construction: the host-side mirror of reference ``utils.py``.

* ``convert_to_matrix``  -- utils.py:10-26 (host, vectorised; the 3-column list is host data).
* ``Adj``                -- the SparseTensor surface the reference touches (``(row, col, value,
  sparse_sizes)`` constructor, ``.to_symmetric()``, ``.storage.rowptr()/col()/value()``,
  utils.py:70-71) plus the device CSR the kernels read: int32, self loops inserted (set_diag).
* ``load_input``         -- utils.py:29-73: the symmetric CSR is built ON THE DEVICE by
  ``hicgat_csr_from_dense`` (a13 + a3), bit-exact with the networkx/to_symmetric pattern.
* ``cont2dist``          -- utils.py:75-80 on the device (``hicgat_cont2dist``, a12).
* ``Truth``              -- the fp32 target of the fused distance/MSE kernel: padded leading dim
  (multiple of 128), symmetric.
"""
import os

import numpy as np
import torch

from . import _lib

TILE = 128


def convert_to_matrix(adj):
    """utils.py:10-26: (bin_i, bin_j, count) list -> dense symmetric matrix, zero rows removed.

    Bins are ranked among the unique ids (``np.argwhere(adj[k,0] == idx)``), later repeats of a
    pair overwrite earlier ones, ``triu(mat) + tril(mat.T, 1)`` is formed exactly as the reference
    does (``tril(., 1)`` also keeps the first super-diagonal, so the diagonal doubles and a list
    with lower-triangle entries gives an asymmetric matrix) and every all-zero column (and the
    same rows) is deleted."""
    adj = np.asarray(adj, dtype=np.float64)
    ids = np.unique(np.concatenate((adj[:, 0], adj[:, 1])))
    mat = np.zeros((len(ids), len(ids)))
    i = np.searchsorted(ids, adj[:, 0])
    j = np.searchsorted(ids, adj[:, 1])
    # last write wins: keep, for every (i, j), the final occurrence in list order
    key = i * len(ids) + j
    _, last = np.unique(key[::-1], return_index=True)
    keep = len(key) - 1 - last
    mat[i[keep], j[keep]] = adj[keep, 2]
    mat = np.triu(mat) + np.tril(mat.T, 1)
    zero = np.argwhere(np.all(mat == 0, axis=0))
    mat = np.delete(mat, zero, axis=1)
    return np.delete(mat, zero, axis=0)


class _Storage:
    def __init__(self, rowptr, col, value):
        self._rowptr, self._col, self._value = rowptr, col, value

    def rowptr(self):
        return self._rowptr

    def col(self):
        return self._col

    def value(self):
        return self._value


class Adj:
    """Symmetric CSR adjacency with a torch_sparse.SparseTensor-like surface.

    ``storage`` holds the reference view (int64, no self loops, row-major sorted/coalesced);
    ``rowptr32``/``col32`` the device view the kernels read (int32, one self loop per row at its
    sorted position, i.e. after PyG's ``set_diag``)."""

    def __init__(self, row=None, col=None, value=None, sparse_sizes=None, *, _csr=None):
        if _csr is not None:
            rowptr, colv, val, n = _csr
        else:
            row = torch.as_tensor(row, dtype=torch.long).cpu()
            colt = torch.as_tensor(col, dtype=torch.long).cpu()
            n = int(sparse_sizes[0]) if sparse_sizes is not None else int(max(row.max(), colt.max())) + 1
            key = row * n + colt
            order = torch.argsort(key, stable=True)
            key = key[order]
            uniq, inverse = torch.unique_consecutive(key, return_inverse=True)
            val = None
            if value is not None:
                v = torch.as_tensor(value)[order]
                val = torch.zeros(uniq.numel(), dtype=v.dtype).index_add(0, inverse, v)
            r = uniq // n
            colv = uniq % n
            rowptr = torch.zeros(n + 1, dtype=torch.long)
            rowptr[1:] = torch.cumsum(torch.bincount(r, minlength=n), 0)
        self.n = n
        self.storage = _Storage(rowptr, colv, val)
        self.rowptr32 = None
        self.col32 = None
        self.value32 = None   # SAGEConv edge weight per device CSR entry (0 on the self loops)
        self.inv_deg = None   # 1 / sum_j w_ij (SAGEConv.adjust_weights, layers.py:41-53)

    def sparse_sizes(self):
        return (self.n, self.n)

    def nnz(self):
        return int(self.storage.col().numel())

    def to_symmetric(self):
        rp, c, v = self.storage.rowptr(), self.storage.col(), self.storage.value()
        r = torch.repeat_interleave(torch.arange(self.n), rp[1:] - rp[:-1])
        vv = None if v is None else torch.cat([v, v])
        return Adj(torch.cat([r, c]), torch.cat([c, r]), vv, (self.n, self.n))

    def to(self, device):
        """Upload the set_diag'd int32 CSR (the host CSR is assumed structurally symmetric)."""
        rp = self.storage.rowptr()
        c = self.storage.col()
        n = self.n
        r = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
        keep = r != c
        r, c = r[keep], c[keep]
        v = self.storage.value()
        r = torch.cat([r, torch.arange(n)])
        c = torch.cat([c, torch.arange(n)])
        key, perm = torch.sort(r * n + c)
        self.rowptr32 = torch.zeros(n + 1, dtype=torch.int32)
        self.rowptr32[1:] = torch.cumsum(torch.bincount(key // n, minlength=n), 0).to(torch.int32)
        self.col32 = (key % n).to(torch.int32)
        if v is not None:
            # the device weights of the self loops are 0; the degree sums run over each row in
            # ascending column order, in float32 (adj_t.sum(dim=0) of a symmetric matrix)
            w = torch.cat([v[keep].float(), torch.zeros(n)])[perm].numpy()
            s = np.zeros(n, dtype=np.float32)
            np.add.at(s, (key // n).numpy(), w)
            with np.errstate(divide="ignore"):
                inv = np.float32(1.0) / s
            self.value32 = torch.tensor(w).to(device)
            self.inv_deg = torch.tensor(inv).to(device)
        self.rowptr32 = self.rowptr32.to(device)
        self.col32 = self.col32.to(device)
        return self

    @property
    def device_nnz(self):
        return int(self.col32.numel())

    @classmethod
    def from_dense_device(cls, A, keep_host=True):
        """a13 + a3 on the GPU: CSR of (A != 0 | A.T != 0), i != j, plus self loops, and the
        networkx edge weights (``value32``) with the SAGEConv normaliser (``inv_deg``).

        ``A`` is a float64 [N, N] device tensor.  The host ``storage`` view (without self loops)
        is derived from the device CSR when ``keep_host`` is set."""
        lib = _lib.lib()
        A = A.contiguous()
        n = A.shape[0]
        dev = A.device
        rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        s = _lib.stream(dev)
        _lib.check(lib.hicgat_csr_from_dense(_lib.ptr(A), n, n, _lib.ptr(rowptr), None, None, 0, s),
                   "hicgat_csr_from_dense(count)")
        nnz = int(rowptr[-1].item())
        col = torch.empty(nnz, dtype=torch.int32, device=dev)
        _lib.check(lib.hicgat_csr_from_dense(_lib.ptr(A), n, n, _lib.ptr(rowptr), _lib.ptr(col), None, 0, s),
                   "hicgat_csr_from_dense(fill)")
        obj = cls.__new__(cls)
        obj.n = n
        obj.rowptr32, obj.col32 = rowptr, col
        obj.value32 = torch.empty(nnz, dtype=torch.float32, device=dev)
        obj.inv_deg = torch.empty(n, dtype=torch.float32, device=dev)
        _lib.check(lib.hicgat_sage_weights(_lib.ptr(A), n, n, _lib.ptr(rowptr), _lib.ptr(col), _lib.ptr(obj.value32),
                                           _lib.ptr(obj.inv_deg), s), "hicgat_sage_weights")
        if keep_host:
            rp = rowptr.cpu().long()
            c = col.cpu().long()
            r = torch.repeat_interleave(torch.arange(n), rp[1:] - rp[:-1])
            keep = r != c
            hrp = torch.zeros(n + 1, dtype=torch.long)
            hrp[1:] = torch.cumsum(torch.bincount(r[keep], minlength=n), 0)
            obj.storage = _Storage(hrp, c[keep], obj.value32.cpu()[keep])
        else:
            obj.storage = None
        return obj


    def tiles(self, min_edges=None):
        """The dense-tile split of the device CSR (``build_tiles``), built once per CSR and cached;
        None when tiling is off (HICGAT_TILE_MIN=0) or, for the default threshold, when the dense
        tiles hold less than TILE_FRAC of the edges."""
        m = TILE_MIN if min_edges is None else int(min_edges)
        if m <= 0:
            return None
        key = (self.rowptr32.data_ptr(), self.col32.data_ptr(), m)
        cache = getattr(self, "_tiles", None)
        if cache is None or cache[0] != key:
            t = build_tiles(self.rowptr32, self.col32, 0, self.n, self.n, m)
            # the tiled form pays where the dense tiles hold nearly every edge (a dense contact map:
            # synth-2000 0.96 vs 1.20 ms per step); on a power-law graph whose tiles hold about half
            # the edges (synth-20000) the gather alone is faster (2.07 vs 2.39 ms per step)
            # (and a graph of a few row blocks, e.g. chr19 1 mb with 58 loci, gains nothing either)
            if min_edges is None and (t.n_dense < TILE_FRAC * self.device_nnz or self.n < TILE_MIN_N):
                t = None
            self._tiles = cache = (key, t)
        return cache[1]


# A 32x32 tile of the contact graph goes to the matrix cores when it holds at least this many
# edges (a dense tile costs the MFMA time of ~64 gathered edges); 0 = off.
TILE_MIN = int(os.environ.get("HICGAT_TILE_MIN", "64"))
# ... and the tiled form is used when the dense tiles hold at least this fraction of the edges
TILE_FRAC = float(os.environ.get("HICGAT_TILE_FRAC", "0.9"))
TILE_MIN_N = int(os.environ.get("HICGAT_TILE_MIN_N", "512"))
TILE_ROWS = 32
TILE_SPLITS = int(os.environ.get("HICGAT_TILE_SPLITS", "0"))   # 0 = from the row-block count


class Tiles:
    """Dense-tile split of rows [r0, r1) of a CSR (include/hicgat.h, hicgat_gat_agg_fwd_tiled):
    ``tptr`` [nrb+1] / ``tcol`` [ntiles] / ``tmask`` [ntiles*32] (int32 bit patterns of uint32
    words) for the row blocks' dense 32x32 tiles, ``rowptr_s`` / ``col_s`` the CSR of every other
    edge; ``n_dense`` edges are in tiles."""

    def __init__(self, r0, r1, tptr, tcol, tmask, rowptr_s, col_s, n_dense, min_edges, max_per_block=0,
                 splits=None):
        self.r0, self.r1 = r0, r1
        self.tptr, self.tcol, self.tmask = tptr, tcol, tmask
        self.rowptr_s, self.col_s = rowptr_s, col_s
        self.ntiles = int(tcol.numel())
        self.n_dense = int(n_dense)
        self.min_edges = min_edges
        # workgroups per row block: enough for ~2 per CU when the graph has few row blocks
        nrb = (r1 - r0 + TILE_ROWS - 1) // TILE_ROWS
        if splits is None:
            splits = TILE_SPLITS or max(1, min(16, max_per_block, -(-512 // max(nrb, 1))))
        self.splits = max(1, min(64, int(splits)))


def build_tiles(rowptr, col, r0, r1, ncols, min_edges=None):
    """Split the edges of rows [r0, r1) of (rowptr, col) into dense 32x32 tiles (row blocks of 32
    from r0, column blocks of 32 from 0) holding >= ``min_edges`` edges, and the CSR of the rest
    (same length as ``rowptr``; rows outside the range empty).  Torch ops on ``col``'s device."""
    m = TILE_MIN if min_edges is None else int(min_edges)
    dev = col.device
    rp = rowptr.long()
    nrb = (r1 - r0 + TILE_ROWS - 1) // TILE_ROWS
    ncb = (ncols + TILE_ROWS - 1) // TILE_ROWS
    beg, end = int(rp[r0]), int(rp[r1])
    deg = rp[r0 + 1:r1 + 1] - rp[r0:r1]
    rows = torch.repeat_interleave(torch.arange(r0, r1, device=dev), deg, output_size=end - beg)
    c = col[beg:end].long()
    key = ((rows - r0) // TILE_ROWS) * ncb + c // TILE_ROWS
    cnt = torch.bincount(key, minlength=nrb * ncb)
    dense = cnt >= max(m, 1)
    in_tile = dense[key]
    tkeys = torch.nonzero(dense).flatten()
    tptr = torch.zeros(nrb + 1, dtype=torch.int64, device=dev)
    tptr[1:] = torch.cumsum(torch.bincount(tkeys // ncb, minlength=nrb), 0)
    tcol = (tkeys % ncb).to(torch.int32)
    tid = torch.searchsorted(tkeys, key[in_tile])
    word = tid * TILE_ROWS + (rows[in_tile] - r0) % TILE_ROWS
    bits = torch.bitwise_left_shift(torch.ones_like(word), c[in_tile] % TILE_ROWS)
    # every (row, col) is one edge: the sum of its distinct bits is their OR
    mask = torch.zeros(tkeys.numel() * TILE_ROWS, dtype=torch.int64, device=dev).index_add_(0, word, bits)
    mask = torch.where(mask >= 2 ** 31, mask - 2 ** 32, mask).to(torch.int32)
    keep = ~in_tile
    n = rp.numel() - 1
    rowptr_s = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    rowptr_s[r0 + 1:r1 + 1] = torch.cumsum(torch.bincount(rows[keep] - r0, minlength=r1 - r0), 0)
    rowptr_s[r1 + 1:] = rowptr_s[r1]
    col_s = c[keep].to(torch.int32)
    if col_s.numel() == 0:
        col_s = torch.zeros(1, dtype=torch.int32, device=dev)   # a valid pointer for an empty remainder
    per = tptr[1:] - tptr[:-1]
    return Tiles(r0, r1, tptr.to(torch.int32), tcol, mask, rowptr_s.to(torch.int32), col_s,
                 int(in_tile.sum()), m, int(per.max()) if nrb > 0 else 0)


class Data:
    """torch_geometric.data.Data stand-in: x, edge_index (Adj), y."""

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)


def load_input(input, features, device="cuda"):
    """utils.py:29-73 with the graph built on the device.

    Returns ``Data(x, edge_index: Adj, y)``; ``y`` is the float64 matrix with zeroed diagonal and
    ``x`` keeps the dtype of ``features`` (utils.py:54), both on ``device``."""
    adj_mat = input
    if adj_mat.shape[1] == 3:
        adj_mat = convert_to_matrix(adj_mat)
    np.fill_diagonal(adj_mat, 0)
    y = torch.tensor(adj_mat, dtype=torch.double, device=device)
    edge_index = Adj.from_dense_device(y)
    x = features.to(device) if isinstance(features, torch.Tensor) else torch.tensor(features).to(device)
    return Data(x=x, edge_index=edge_index, y=y)


def cont2dist(adj, factor, dtype=torch.float64):
    """utils.py:75-80 on the device: (1/y)^f, diag 0, +inf -> max finite, NaN -> 0, / max."""
    lib = _lib.lib()
    y = adj.to(torch.float64).contiguous()
    n = y.shape[0]
    out = torch.empty((n, n), dtype=dtype, device=y.device)
    ws = _lib.workspace(lib.hicgat_cont2dist_workspace_bytes(n), y.device)
    o32 = out if dtype == torch.float32 else None
    o64 = out if dtype == torch.float64 else None
    _lib.check(lib.hicgat_cont2dist(_lib.ptr(y), n, n, float(factor), _lib.ptr(o32), _lib.ptr(o64), n,
                                    _lib.ptr(ws), ws.numel(), _lib.stream(y.device)), "hicgat_cont2dist")
    return out


def padded_ld(n):
    return ((n + TILE - 1) // TILE) * TILE


# The fused loss takes the truth in background + support form when the entries that differ from
# the background are at most this fraction of the matrix (HICGAT_TRUTH_SUPPORT=0: always dense).
SUPPORT_BACKGROUND = 1.0 if os.environ.get("HICGAT_TRUTH_SUPPORT", "1") != "0" else None
SUPPORT_MAX_FRACTION = 0.25


class SupportForm:
    """A symmetric truth as ``background`` off the diagonal except at a sorted CSR support
    (``rowptr``, ``col``, ``val``: the entries that differ, no diagonal) plus ``diag``.
    ``cont2dist``'s target (utils.py:75-80) is 1 wherever the contact count is 0 (inf -> max ->
    /max), so its support is the contact set: the fused loss then streams no truth
    (hicgat_pairdist_mse_fused_support).  Built on the device by hicgat_truth_support from the
    stored (symmetrised) truth, so the values are the dense ones, bit for bit."""

    def __init__(self, background, rowptr, col, val, diag, nnz):
        # col / val hold at least one element (a non-null pointer for an empty support)
        self.background, self.rowptr, self.col_buf, self.val_buf, self.diag = background, rowptr, col, val, diag
        self.nnz = nnz

    @property
    def col(self):
        return self.col_buf[:self.nnz]

    @property
    def val(self):
        return self.val_buf[:self.nnz]

    @classmethod
    def build(cls, truth, background, max_fraction=SUPPORT_MAX_FRACTION):
        """The form, or None when the support is denser than ``max_fraction`` of the matrix."""
        lib = _lib.lib()
        n, dev = truth.n, truth.buf.device
        st = _lib.stream(dev)
        rowptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
        _lib.check(lib.hicgat_truth_support(_lib.ptr(truth.buf), n, truth.ld, float(background), _lib.ptr(rowptr),
                                            None, None, None, st), "hicgat_truth_support")
        # int32 counts: a wrap past 2^31 shows as a negative step
        if bool((rowptr[1:] < rowptr[:-1]).any()):
            return None
        nnz = int(rowptr[-1])
        if nnz > max_fraction * float(n) * float(n):
            return None
        col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
        val = torch.empty(max(nnz, 1), dtype=torch.float32, device=dev)
        diag = torch.empty(n, dtype=torch.float32, device=dev)
        _lib.check(lib.hicgat_truth_support(_lib.ptr(truth.buf), n, truth.ld, float(background), _lib.ptr(rowptr),
                                            _lib.ptr(col), _lib.ptr(val), _lib.ptr(diag), st),
                   "hicgat_truth_support")
        return cls(float(background), rowptr, col, val, diag, nnz)

    @classmethod
    def build_host(cls, truth, background, max_fraction=SUPPORT_MAX_FRACTION):
        """The same form of a CPU truth (torch ops; the multi-rank CPU tests), or None."""
        n = truth.n
        t = truth.buf[:, :n].float()
        off = (t != float(background)) & ~torch.eye(n, dtype=torch.bool)
        nnz = int(off.sum())
        if nnz > max_fraction * float(n) * float(n):
            return None
        rows, cols = off.nonzero(as_tuple=True)
        rowptr = torch.zeros(n + 1, dtype=torch.int64)
        rowptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
        col = cols.to(torch.int32) if nnz else torch.zeros(1, dtype=torch.int32)
        val = t[rows, cols].contiguous() if nnz else torch.zeros(1)
        return cls(float(background), rowptr.to(torch.int32), col, val, t.diagonal().contiguous(), nnz)


class Truth:
    """fp32 target for the fused distance/MSE kernel: [N, ld] with ld = ceil(N/128)*128.

    ``Truth.from_contacts(y, factor)`` runs cont2dist straight into the padded buffer;
    ``Truth(t)`` copies an existing [N, N] target (``truth.float()`` of the reference loop).

    The fused kernel reads only the upper-triangle tiles (one T read per pair).  A target that is
    not exactly symmetric -- R's KR scaling forms (x_i A_ij) x_j and (x_j A_ji) x_i, which can round
    apart (r_utils.R:74-89), and the reference's MSELoss simply proceeds -- is stored in the
    equivalent symmetric form: for every pair, with d_ij = d_ji and tbar = (T_ij + T_ji)/2,
      (d - T_ij)^2 + (d - T_ji)^2 = 2 (d - tbar)^2 + (T_ij - T_ji)^2 / 2,
    so the off-diagonal becomes tbar (same gradient) and the constant (T_ij - T_ji)^2 / 2 of row i's
    pairs j > i is folded into the diagonal, whose only role is the (0 - T_ii)^2 term of the MSE
    (cdist's diagonal is 0 and carries no gradient): T'_ii = sqrt(T_ii^2 + sum_j>i (T_ij - T_ji)^2/2).
    The MSE value and its gradient are unchanged (to fp32 rounding); ``asymmetric_source`` records it
    and ``scoring()`` keeps the target as given for dSCC (the reference ranks truth[triu] itself).
    The combined loss's Pearson term then sees tbar on the upper triangle (a relative change of
    the order of the asymmetry, 1e-7 for R's rounding)."""

    def __init__(self, t=None, *, _buf=None, _n=None, background=SUPPORT_BACKGROUND):
        if _buf is None:
            t = t.detach()
            n = t.shape[0]
            buf = torch.zeros((n, padded_ld(n)), dtype=torch.float32, device=t.device)
            buf[:, :n] = t.float()
        else:
            buf, n = _buf, _n
        self.buf, self.n, self.ld = buf, n, buf.shape[1]
        view = buf[:, :n]
        self.asymmetric_source = not bool(torch.equal(view, view.t()))
        self.raw = None
        if self.asymmetric_source:
            # the target as given, kept on the HOST (scoring() is read once per run; a device copy would
            # double the truth's HBM for the whole run): dSCC scores its upper triangle
            self.raw = view.to("cpu", copy=True)
            self._symmetrise()
        self.symmetric = True
        self.support = None
        if background is not None and buf.is_cuda and n > 1:
            self.support = SupportForm.build(self, background)

    def _symmetrise(self):
        t = self.buf[:, :self.n].double()
        diff2 = torch.triu((t - t.t()) ** 2, 1).sum(1) * 0.5
        sym = (t + t.t()) * 0.5
        sym.diagonal().copy_(torch.sqrt(t.diagonal() ** 2 + diff2))
        self.buf[:, :self.n] = sym.float()

    @classmethod
    def from_contacts(cls, y, factor):
        lib = _lib.lib()
        y = y.to(torch.float64).contiguous()
        n = y.shape[0]
        ld = padded_ld(n)
        buf = torch.zeros((n, ld), dtype=torch.float32, device=y.device)
        ws = _lib.workspace(lib.hicgat_cont2dist_workspace_bytes(n), y.device)
        _lib.check(lib.hicgat_cont2dist(_lib.ptr(y), n, n, float(factor), _lib.ptr(buf), None, ld,
                                        _lib.ptr(ws), ws.numel(), _lib.stream(y.device)),
                   "hicgat_cont2dist")
        return cls(_buf=buf, _n=n)

    def dense(self):
        return self.buf[:, :self.n]

    def upper(self):
        """The target the contrastive loss sees: truth[triu] AS GIVEN in both triangles (that loss reads
        the upper-triangle entries themselves, not their symmetric mean) -- ``self`` when the source was
        symmetric; otherwise a second Truth, built once and cached."""
        if self.raw is None:
            return self
        if getattr(self, "_upper", None) is None:
            t = self.raw.to(self.buf.device)
            u = torch.triu(t, 1)
            self._upper = Truth(u + u.t(), background=None if self.support is None else self.support.background)
        return self._upper

    def scoring(self):
        """The matrix whose upper triangle the reference scores dSCC against (HiC-GNN_main.py:135-139
        takes truth[triu] as given): the target before symmetrisation when it was asymmetric."""
        return self.raw.to(self.buf.device) if self.raw is not None else self.dense()
