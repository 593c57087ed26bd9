"""GPU: node2vec -- the HIP walks against the exact node2vec transition
table of oracle/node2vec.py, and the HIP skip-gram's embeddings on graphs with known structure.
Parity for the embeddings is unpinned (no reference embeddings ship); the walk
distribution is checked statistically (total-variation distance of empirical transition
frequencies, tolerance sized for the sample counts)."""
import collections

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


def _weighted(n=14, seed=3):
    rng = np.random.default_rng(seed)
    a = rng.random((n, n)) * (rng.random((n, n)) < 0.45) * 3 + 0.0
    a = np.triu(a, 1)
    a = a + a.T
    for i in range(n - 1):                    # connected
        a[i, i + 1] = a[i + 1, i] = max(a[i, i + 1], 0.5)
    a[2, 2] = 0.8                              # a self loop
    return a


def test_walks_valid_deterministic_and_shuffled_rounds():
    from hicgat import embed
    from oracle import node2vec as on
    a = _weighted(40, 1)
    a[7, :] = a[:, 7] = 0                      # isolated node: its walks stop at once
    rowptr, col, _ = on.graph_csr(a)
    w1 = embed.random_walks(a, num_walks=6, walk_length=30, p=0.5, q=2.0, seed=7).cpu().numpy()
    w2 = embed.random_walks(a, num_walks=6, walk_length=30, p=0.5, q=2.0, seed=7).cpu().numpy()
    w3 = embed.random_walks(a, num_walks=6, walk_length=30, p=0.5, q=2.0, seed=8).cpu().numpy()
    assert np.array_equal(w1, w2) and not np.array_equal(w1, w3)
    n = a.shape[0]
    for r in range(6):                         # every round starts one walk from every node
        assert sorted(w1[r * n:(r + 1) * n, 0]) == list(range(n))
    adj = {i: set(col[rowptr[i]:rowptr[i + 1]]) for i in range(n)}
    for walk in w1:
        if walk[0] == 7:
            assert (walk[1:] == -1).all()
            continue
        assert (walk >= 0).all()
        for u, v in zip(walk[:-1], walk[1:]):
            assert v in adj[u]


def test_walk_transition_frequencies_match_node2vec_table():
    """Second-order steps (prev, cur) -> next and first steps cur -> next against the exact tables."""
    from hicgat import embed
    from oracle import node2vec as on
    a = _weighted()
    p, q = 0.5, 2.5
    rowptr, col, w = on.graph_csr(a)
    walks = embed.random_walks(a, num_walks=4000, walk_length=6, p=p, q=q, seed=11).cpu().numpy()
    first = collections.defaultdict(collections.Counter)
    second = collections.defaultdict(collections.Counter)
    for walk in walks:
        first[walk[0]][walk[1]] += 1
        for t in range(2, walk.shape[0]):
            second[(walk[t - 2], walk[t - 1])][walk[t]] += 1
    checked = 0
    for cur, cnt in first.items():
        nb, pr = on.first_step(rowptr, col, w, cur)
        tot = sum(cnt.values())
        emp = np.array([cnt[k] for k in nb]) / tot
        assert 0.5 * np.abs(emp - pr).sum() < 2.0 / np.sqrt(tot) + 0.01, cur
        checked += 1
    for (prev, cur), cnt in second.items():
        tot = sum(cnt.values())
        if tot < 2000:
            continue
        nb, pr = on.second_step(rowptr, col, w, prev, cur, p, q)
        emp = np.array([cnt[k] for k in nb]) / tot
        assert set(cnt) <= set(nb)
        assert 0.5 * np.abs(emp - pr).sum() < 2.0 / np.sqrt(tot) + 0.01, (prev, cur)
        checked += 1
    assert checked > 40


def test_skipgram_separates_planted_communities():
    """Two dense communities joined by a few weak edges: after node2vec, nodes are closer (cosine)
    to their own community than to the other one; the embeddings are finite and of the asked shape."""
    from hicgat import embed
    rng = np.random.default_rng(0)
    n = 40
    a = np.zeros((n, n))
    for lo, hi in ((0, 20), (20, 40)):
        blk = rng.random((hi - lo, hi - lo)) * (rng.random((hi - lo, hi - lo)) < 0.6) + 0.1
        a[lo:hi, lo:hi] = np.triu(blk, 1) + np.triu(blk, 1).T
    for i, j in ((0, 20), (5, 31), (13, 27)):
        a[i, j] = a[j, i] = 0.05
    np.fill_diagonal(a, 0)
    emb = embed.node2vec(a, dimensions=64, walk_length=40, num_walks=20, p=1.0, q=1.0, window=5, epochs=3,
                         seed=1).cpu().numpy()
    assert emb.shape == (n, 64) and np.isfinite(emb).all()
    e = emb / np.linalg.norm(emb, axis=1, keepdims=True)
    cos = e @ e.T
    lab = np.arange(n) < 20
    same = cos[lab[:, None] == lab[None, :]]
    diff = cos[lab[:, None] != lab[None, :]]
    assert same.mean() > diff.mean() + 0.2, (same.mean(), diff.mean())


def test_node2vec_reference_call_on_chr19():
    """The reference's own call (dimensions 512, walk_length 150, num_walks 50, p 1.75, q 0.4,
    window 25, 5 epochs) on the chr19 1 mb contacts: shape, finiteness, and neighbouring loci
    (the Hi-C diagonal) more similar than distant ones."""
    from conftest import load_golden
    from hicgat import embed
    a = load_golden("graph_chr19_1mb.npz")["matrix"].copy()
    emb = embed.node2vec(a).cpu().numpy()
    n = a.shape[0]
    assert emb.shape == (n, 512) and np.isfinite(emb).all()
    e = emb / np.linalg.norm(emb, axis=1, keepdims=True)
    cos = e @ e.T
    near = np.mean([cos[i, i + 1] for i in range(n - 1)])
    far = np.mean([cos[i, j] for i in range(n) for j in range(n) if abs(i - j) > n // 3])
    assert near > far, (near, far)
