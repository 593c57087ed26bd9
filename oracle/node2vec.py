"""Oracle: node2vec walk distributions and gensim Word2Vec tables (TEST INFRASTRUCTURE ONLY).

Restates, from their published code (neither package is installed):

* ``graph_csr``       -- networkx ``from_numpy_matrix(A)`` (HiC_GAT_generalize_directly.py:150):
                         an undirected Graph built row by row, so edge {i, j} exists when A[i, j] or
                         A[j, i] is non-zero (self loops included) and the later (max, min)
                         assignment overwrites the weight; pinned against networkx itself
                         (tests/test_oracle_golden.py).
* ``first_step`` / ``second_step`` -- node2vec 0.4.x ``Node2Vec._precompute_probabilities``: from
                         cur, after prev, neighbour d of cur gets weight w(cur, d) / p if d == prev,
                         w(cur, d) if d is a neighbour of prev, w(cur, d) / q otherwise, normalised;
                         the first step uses w(cur, d) alone.
* ``downsample_keep`` / ``cum_table`` -- gensim 4 ``Word2Vec.prepare_vocab`` (sample = 1e-3) and
                         ``make_cum_table`` (ns_exponent 0.75, domain 2^31 - 1).

Parity unpinned for the embeddings themselves: the reference ships no embedding files (SURVEY 8(f)
row f4); tests check the GPU walks' empirical transition frequencies against these exact tables and
the structure of the learned embeddings.
"""
import numpy as np


def graph_csr(A):
    """Sorted CSR (rowptr, col, weight) of ``networkx.from_numpy_matrix(A)``; NaN entries are no edge."""
    A = np.nan_to_num(np.asarray(A, dtype=np.float64), nan=0.0)
    n = A.shape[0]
    lo = np.tril(A, -1)
    up = np.triu(A, 1).T                        # up[i, j] = A[j, i] for i > j
    wl = np.where(lo != 0, lo, up)              # the weight networkx keeps for the pair (i > j)
    W = wl + wl.T + np.diag(np.diag(A))
    rows, cols = np.nonzero(W)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, rows + 1, 1)
    return np.cumsum(rowptr), cols.astype(np.int64), W[rows, cols]


def first_step(rowptr, col, w, cur):
    s, e = rowptr[cur], rowptr[cur + 1]
    ww = w[s:e]
    return col[s:e], ww / ww.sum()


def second_step(rowptr, col, w, prev, cur, p, q):
    s, e = rowptr[cur], rowptr[cur + 1]
    nb, ww = col[s:e], w[s:e]
    prev_nb = col[rowptr[prev]:rowptr[prev + 1]]
    f = np.where(nb == prev, 1.0 / p, np.where(np.isin(nb, prev_nb), 1.0, 1.0 / q))
    pr = ww * f
    return nb, pr / pr.sum()


def downsample_keep(counts, sample=1e-3):
    counts = np.asarray(counts, dtype=np.float64)
    thr = sample * counts.sum()
    with np.errstate(divide="ignore", invalid="ignore"):
        p = (np.sqrt(counts / thr) + 1.0) * (thr / counts)
    return np.where(counts > 0, np.minimum(p, 1.0), 0.0)


def cum_table(counts, ns_exponent=0.75, domain=2 ** 31 - 1):
    pw = np.asarray(counts, dtype=np.float64) ** ns_exponent
    return np.round(np.cumsum(pw) / pw.sum() * domain).astype(np.uint32)
