"""Oracle: Hi-C list -> matrix -> CSR graph -> distance target (TEST INFRASTRUCTURE ONLY).

Restates reference ``utils.py`` (``convert_to_matrix`` :10-26, ``load_input`` :29-73,
``cont2dist`` :75-80) plus the torch_sparse 0.6.11 ``SparseTensor.to_symmetric`` (sort + coalesce,
sum reduce) and ``set_diag`` behaviour that PyG 1.7.2 ``GATConv`` applies (un-vendored; restated
from the published algorithm).
"""
import numpy as np
import torch


def convert_to_matrix(adj):
    """Restates ``utils.py:10-26``.

    ``adj`` is an (L, 3) array of ``(bin_i, bin_j, count)``.  Bins are mapped to their rank among
    the unique bin ids, the last write wins for repeated pairs (the reference loop order), the
    upper triangle is mirrored (``triu + tril(T, 1)``; the diagonal is *not* doubled by that sum
    because ``tril(., 1)`` excludes it) and all-zero columns (and the same rows) are removed.
    """
    adj = np.asarray(adj, dtype=np.float64)
    ids = np.unique(np.concatenate((adj[:, 0], adj[:, 1])))
    size = len(ids)
    mat = np.zeros((size, size))
    i = np.searchsorted(ids, adj[:, 0])
    j = np.searchsorted(ids, adj[:, 1])
    # sequential assignment keeps "last write wins" exactly like utils.py:17-20
    for k in range(len(adj)):
        mat[i[k], j[k]] = adj[k, 2]
    mat = np.triu(mat) + np.tril(mat.T, 1)
    zero_cols = np.argwhere(np.all(mat[..., :] == 0, axis=0))
    mat = np.delete(mat, zero_cols, axis=1)
    mat = np.delete(mat, zero_cols, axis=0)
    return mat


def csr_from_matrix(adj):
    """Symmetric off-diagonal CSR of ``adj != 0`` (``utils.py:33-71``).

    ``nx.from_numpy_array(adj).to_undirected()`` creates one undirected edge for every (i, j) with
    ``adj[i, j] != 0`` or ``adj[j, i] != 0``; self loops are masked (``:59-63``); ``SparseTensor(...)
    .to_symmetric()`` adds the reverse direction and coalesces into row-major sorted CSR.  The edge
    value is the networkx weight: entries are inserted in row-major order, so for i < j the later
    ``adj[j, i]`` (when non-zero) overwrites ``adj[i, j]``; the value is cast to float32 (``:52``).

    Returns ``(rowptr int64 [N+1], col int64 [nnz], value float32 [nnz])``.
    """
    a = np.array(adj, dtype=np.float64, copy=True)
    np.fill_diagonal(a, 0)
    n = a.shape[0]
    nz = a != 0
    pattern = nz | nz.T
    np.fill_diagonal(pattern, False)
    upper_w = np.where(nz.T, a.T, a)          # weight of edge (i<j): adj[j,i] if non-zero else adj[i,j]
    w = np.where(np.triu(np.ones((n, n), dtype=bool), 1), upper_w, upper_w.T).astype(np.float32)
    rows, cols = np.nonzero(pattern)          # row-major == coalesced sorted order
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, rows + 1, 1)
    rowptr = np.cumsum(rowptr)
    return rowptr, cols.astype(np.int64), w[rows, cols]


def set_diag(rowptr, col):
    """torch_sparse ``set_diag`` (no values): insert (i, i) into every row at its sorted position.

    PyG 1.7.2 ``GATConv.forward`` calls it on a SparseTensor ``edge_index`` when
    ``add_self_loops=True``.  Any existing diagonal entry is removed first (``remove_diag``).
    """
    rowptr = np.asarray(rowptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    n = len(rowptr) - 1
    row = np.repeat(np.arange(n), np.diff(rowptr))
    keep = row != col
    row, col = row[keep], col[keep]
    row = np.concatenate((row, np.arange(n)))
    col = np.concatenate((col, np.arange(n)))
    order = np.lexsort((col, row))
    row, col = row[order], col[order]
    new_ptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(new_ptr, row + 1, 1)
    return np.cumsum(new_ptr), col


def load_input(matrix, features):
    """Restates ``utils.load_input`` (``utils.py:29-73``) without torch_geometric.

    Returns a dict with ``x`` (tensor of ``features`` in its own dtype, ``:54``), ``rowptr``/``col``
    (int64 CSR, symmetric, no self loops) and ``y`` (float64 matrix with zeroed diagonal, ``:33-35``).
    Like the reference, a 3-column input is converted with ``convert_to_matrix`` first and the
    diagonal of ``matrix`` is zeroed in place.
    """
    adj = matrix
    if adj.shape[1] == 3:
        adj = convert_to_matrix(adj)
    np.fill_diagonal(adj, 0)
    y = torch.tensor(adj, dtype=torch.double)
    rowptr, col, value = csr_from_matrix(adj)
    return {"x": torch.tensor(features), "rowptr": rowptr, "col": col, "value": value, "y": y}


def cont2dist(adj, factor):
    """Restates ``utils.py:75-80``: (1/y)^f, zero diagonal, +inf -> max finite value, / max."""
    dist = (1 / adj) ** factor
    dist.fill_diagonal_(0)
    mx = torch.max(torch.nan_to_num(dist, posinf=0))
    dist = torch.nan_to_num(dist, posinf=mx)
    return dist / mx
