"""The shards the driver's multi-GPU bench uses: ``hicgat.dist.ShardPlan`` on the synth-20000 graph
(BASELINE configs[2] / [3], N = 20000, 4.02 M CSR entries with self loops) for P = 2 ... 8, host
only.  Every upper-triangle loss tile is owned exactly once, each rank's dense truth band covers
its tiles, per-rank nnz is within 2 % of nnz / P, the support rows partition the contact set, and
every rank's local CSRs map back to the global CSR (both step forms)."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from hicgat import synth  # noqa: E402
from hicgat.dist import TILE, ShardPlan, partition_rows, tri_row  # noqa: E402


@pytest.fixture(scope="module")
def synth20000():
    n = 20000
    i, j, _ = synth.contact_pairs(n, density=0.01, seed=0)
    # the symmetric CSR with self loops (set_diag), rows sorted -- what Adj builds on the device
    rows = np.concatenate([i, j, np.arange(n)])
    cols = np.concatenate([j, i, np.arange(n)])
    order = np.lexsort((cols, rows))
    rows, cols = rows[order], cols[order]
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=rowptr[1:])
    # the loss support of cont2dist's target: the contacts (no diagonal)
    off = rows != cols
    srp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows[off], minlength=n), out=srp[1:])
    return rowptr, cols, srp


@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8])
def test_synth20000_plan(synth20000, P):
    rowptr, col, srp = synth20000
    n, nnz = rowptr.shape[0] - 1, int(rowptr[-1])
    assert nnz > 4_000_000
    plan = ShardPlan(rowptr, col, P, support_rowptr=srp)
    # rows: contiguous, every rank non-empty, nnz within 2 % of nnz / P
    assert plan.bounds[0] == 0 and plan.bounds[-1] == n and (np.diff(plan.bounds) >= 1).all()
    assert plan.nnz.sum() == nnz
    assert np.abs(plan.nnz - nnz / P).max() <= 0.02 * nnz / P, plan.nnz
    # support rows: a partition of the contact set, balanced
    assert plan.sbounds[0] == 0 and plan.sbounds[-1] == n and plan.snnz.sum() == srp[-1]
    assert np.abs(plan.snnz - srp[-1] / P).max() <= 0.02 * srp[-1] / P, plan.snnz
    # tiles: the ranges partition [0, tiles) -- every upper-triangle tile owned exactly once
    owned = np.zeros(plan.tiles, dtype=np.int64)
    for r in range(P):
        t0, t1 = plan.tile_range(r)
        owned[t0:t1] += 1
        if t1 > t0:
            # the rank's dense truth band covers every row / column its tiles read
            b0, b1, c0 = plan.truth_band(r)
            nb = plan.nb
            for t in (t0, (t0 + t1) // 2, t1 - 1):
                I = tri_row(t, nb)
                J = I + (t - (I * nb - I * (I - 1) // 2))
                assert I <= J < nb
                assert b0 <= I * TILE and min(n, (I + 1) * TILE) <= b1 and c0 <= J * TILE
            assert tri_row(t0, nb) * TILE == b0
    assert (owned == 1).all()
    # local CSRs map back to the global CSR
    inv = np.empty(P * plan.R, dtype=np.int64)
    inv[plan.gidx] = np.arange(n)
    slab_total = 0
    slab_rows = np.zeros(n, dtype=np.int64)
    for r in range(P):
        r0, r1, q0 = plan.rows(r)
        e0, e1 = rowptr[r0], rowptr[r1]
        rp, cl = plan.local_csr(r)                    # "allgather" form: buffer numbering
        assert rp[q0] == 0 and rp[q0 + (r1 - r0)] == e1 - e0 and rp[-1] == e1 - e0
        assert np.array_equal(inv[cl], col[e0:e1])
        rp, cl = plan.own_csr(r)                      # "slab" form, forward: global numbering
        assert np.array_equal(rp[r0:r1 + 1], rowptr[r0:r1 + 1] - e0) and np.array_equal(cl, col[e0:e1])
        rp, cl = plan.slab_csr(r)                     # "slab" form, source pass
        assert ((cl >= r0) & (cl < r1)).all()
        slab_total += cl.shape[0]
        slab_rows += np.diff(rp.astype(np.int64))
        # row r's slab entries are exactly its CSR neighbours owned by this rank, in order
        for g in (0, r0, r1 - 1, n // 2, n - 1):
            nbrs = col[rowptr[g]:rowptr[g + 1]]
            assert np.array_equal(cl[rp[g]:rp[g + 1]], nbrs[(nbrs >= r0) & (nbrs < r1)])
    assert slab_total == nnz and np.array_equal(slab_rows, np.diff(rowptr))


def test_partition_keeps_every_rank_nonempty_on_a_hub_graph():
    """one hub row holding most of the edges put two cuts on the same row; the cuts
    are clamped so every rank keeps at least one row."""
    deg = np.ones(40, dtype=np.int64)
    deg[3] = 10_000                                  # a hub row: > nnz / P for every P here
    rp = np.concatenate([[0], np.cumsum(deg)])
    for P in range(2, 9):
        b = partition_rows(rp, P)
        assert b[0] == 0 and b[-1] == 40 and (np.diff(b) >= 1).all(), (P, b)
    with pytest.raises(ValueError, match="at least one row"):
        ShardPlan(np.arange(4), np.arange(3), 4)
