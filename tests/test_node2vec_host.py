"""CPU: the node2vec host side -- the weighted graph (networkx's from_numpy_matrix rule, pinned
against networkx itself), the second-order transition table, gensim's vocabulary tables -- product
(hicgat.embed) vs oracle (oracle/node2vec.py)."""
import numpy as np
import pytest

from conftest import load_golden


def _weighted(n=30, seed=0):
    rng = np.random.default_rng(seed)
    a = rng.random((n, n)) * (rng.random((n, n)) < 0.3)
    a[3, 7], a[7, 3] = 0.0, 2.5           # asymmetric: only the lower entry set
    a[9, 2], a[2, 9] = 1.5, 0.0           # only the upper entry set
    a[4, 4] = 0.7                          # a self loop
    a[11, :] = a[:, 11] = 0.0              # an isolated node
    return a


@pytest.mark.parametrize("case", ["weighted", "chr19_1mb"])
def test_graph_csr_matches_networkx(case):
    nx = pytest.importorskip("networkx")
    from oracle import node2vec as on
    a = _weighted() if case == "weighted" else load_golden("graph_chr19_1mb.npz")["matrix"].copy()
    G = nx.from_numpy_array(a)              # from_numpy_matrix of networkx < 3
    rowptr, col, w = on.graph_csr(a)
    n = a.shape[0]
    for i in range(n):
        nb = sorted(G.neighbors(i))
        assert list(col[rowptr[i]:rowptr[i + 1]]) == nb
        assert np.array_equal(w[rowptr[i]:rowptr[i + 1]], [G[i][j]["weight"] for j in nb])


def test_product_host_tables_equal_oracle():
    from hicgat import embed
    from oracle import node2vec as on
    a = _weighted(40, 1)
    for x, y in zip(embed.graph_csr(a), on.graph_csr(a)):
        assert np.array_equal(x, y)
    counts = np.random.default_rng(2).integers(0, 5000, 40)
    keep, cum = embed.vocab_tables(counts)
    assert np.allclose(keep, on.downsample_keep(counts), rtol=1e-6)
    assert np.array_equal(cum, on.cum_table(counts))
    assert cum[-1] == 2 ** 31 - 1


def test_second_step_table_factors():
    """The table's three cases on a hand-built graph: back to prev (1/p), a neighbour of prev (1),
    farther (1/q)."""
    from oracle import node2vec as on
    a = np.zeros((4, 4))
    for i, j, v in ((0, 1, 1.0), (1, 2, 2.0), (1, 3, 1.0), (0, 2, 1.0)):
        a[i, j] = a[j, i] = v
    rowptr, col, w = on.graph_csr(a)
    nb, pr = on.second_step(rowptr, col, w, prev=0, cur=1, p=0.5, q=4.0)
    raw = {0: 1.0 / 0.5, 2: 2.0, 3: 1.0 / 4.0}       # 2 is adjacent to 0, 3 is not
    tot = sum(raw.values())
    assert list(nb) == [0, 2, 3]
    assert np.allclose(pr, [raw[k] / tot for k in nb])


def test_initial_vectors_follow_gensim4_prep_vectors():
    """gensim 4 ``prep_vectors``: default_rng(seed).random((V, D)) * 2 - 1, / D, rows in the
    vocabulary order of sort_by_descending_frequency (np.argsort(count)[::-1] over the words in
    first-appearance order: ties come out reversed); Word2Vec's default seed 1."""
    import torch
    from hicgat import embed
    walks = torch.tensor([[2, 0, 2, 1, -1], [3, 2, 0, 0, 2]], dtype=torch.int32)   # counts 0:3 1:1 2:4 3:1
    v = embed.initial_vectors(walks, 5, 8, w2v_seed=1)
    ref = np.random.default_rng(seed=1).random((4, 8), dtype=np.float32) * 2.0 - 1.0
    ref /= 8
    scan, cnt = np.array([2, 0, 1, 3]), np.array([4, 3, 1, 1])     # first appearance; counts 4, 3, 1, 1
    order = list(scan[np.argsort(cnt)[::-1]])
    assert order[:2] == [2, 0]            # 2 (4x), 0 (3x), then the tie 1 / 3 in numpy's argsort order
    for rank, node in enumerate(order):
        assert np.array_equal(v[node], ref[rank])
    assert not v[4].any()                 # never visited: not in the vocabulary
    assert np.abs(v[:4]).max() < 1.0 / 8


@pytest.mark.parametrize("fixture", ["n2v_chr19_1mb.npz", "n2v_chr19_1mb_s43.npz"])
def test_node2vec_chr19_embedding_structure(fixture):
    """BASELINE configs[0]'s 512-d node2vec features (this repo's GPU node2vec with the reference's
    parameters, seeds 42 and 43, tests/golden/make_n2v_chr19.py): the embedding is dominated by one
    common direction -- the shift of skip-gram's implicit shifted-PMI factorisation on a 58-word,
    fully co-occurring vocabulary -- with the genomic structure in the small centred remainder.
    Measured and pinned here (why config 0's dSCC collapses on both sides)."""
    from hicgat import embed
    from oracle import graph as ogr
    from oracle import kr as okr
    x = np.asarray(load_golden(fixture)["x"], dtype=np.float32)
    a = np.array(load_golden("graph_chr19_1mb.npz")["matrix"], dtype=np.float64)
    np.fill_diagonal(a, 0)
    normed, _ = okr.krnorm(a.copy())
    t = ogr.cont2dist(ogr.load_input(normed.copy(), x)["y"], 0.5).numpy()
    st = embed.embedding_stats(x, t)
    print(fixture, {k: round(v, 4) for k, v in st.items()})
    assert st["shared"] > 0.95 and st["cos_mean"] > 0.95      # common-component dominated
    assert st["locality"] > 0.2 and st["truth_rho"] > 0.5     # the structure is in the centred remainder
