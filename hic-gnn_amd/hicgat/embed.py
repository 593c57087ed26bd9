"""node2vec embeddings on the GPU.

Reference call (HiC_GAT_generalize_directly.py:150-155; the same at evaluate_combined_loss.py:78 and
HiC-GNN_node2vec_conversion.py:118 with other p / q / walk lengths):

    G = nx.from_numpy_matrix(matrix)
    Node2Vec(G, dimensions=512, walk_length=150, num_walks=50, p=1.75, q=0.4, workers=1, seed=42)
        .fit(window=25, min_count=1, batch_words=4)      # gensim Word2Vec, sg=1
    embeddings = [model.wv[str(node)] for node in G.nodes()]

``node2vec(matrix, ...)`` returns the [N, dimensions] embedding matrix in node order.  The walks
(``hicgat_n2v_walks``) and the skip-gram epochs (``hicgat_n2v_sgns_epoch``) run in libhicgat.so;
the host builds the weighted CSR (networkx's edge / weight rule) and gensim's vocabulary tables
(downsampling keep probabilities, unigram^0.75 negative-sampling table) from the walk counts.
Differences from the reference, by construction: the random streams of the walks and of the
skip-gram (a counter-based RNG instead of Python's / gensim's LCG) and the update order of the
concurrent skip-gram waves (``max_waves``; the reference trains with one worker) -- node2vec output
is stochastic, so no two implementations agree bit for bit.  The initial vectors are gensim 4's
(``initial_vectors``: same generator, same vocabulary order, given the walks).
"""
import numpy as np
import torch

from . import _lib

P = _lib.ptr


def graph_csr(A):
    """Sorted CSR (rowptr, col, weight) of ``networkx.from_numpy_matrix(A)``: edge {i, j} when
    A[i, j] or A[j, i] is non-zero (self loops included), weight A[max, min] if non-zero else
    A[min, max] (the undirected Graph keeps the later assignment); NaN entries are no edge."""
    A = np.nan_to_num(np.asarray(A, dtype=np.float64), nan=0.0)
    n = A.shape[0]
    lo = np.tril(A, -1)
    wl = np.where(lo != 0, lo, np.triu(A, 1).T)
    W = wl + wl.T + np.diag(np.diag(A))
    rows, cols = np.nonzero(W)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, rows + 1, 1)
    return np.cumsum(rowptr), cols.astype(np.int64), W[rows, cols]


def random_walks(A, num_walks=50, walk_length=150, p=1.75, q=0.4, seed=42, device="cuda"):
    """[num_walks * N, walk_length] int32 walks (-1 padded): num_walks rounds, each starting one walk
    from every node in a shuffled order (node2vec's ``_generate_walks``)."""
    lib = _lib.lib()
    rowptr, col, w = graph_csr(A)
    n = len(rowptr) - 1
    # inclusive per-row cumulative weights (float64 prefix sums, stored as float32)
    cs = np.cumsum(w)
    base = np.repeat(np.concatenate([[0.0], cs])[rowptr[:-1]], np.diff(rowptr))
    cumw = (cs - base).astype(np.float32)
    rng = np.random.default_rng(seed)
    starts = np.concatenate([rng.permutation(n) for _ in range(num_walks)]).astype(np.int32)
    dev = torch.device(device)
    t_rowptr = torch.tensor(rowptr, dtype=torch.int32, device=dev)
    t_col = torch.tensor(col, dtype=torch.int32, device=dev)
    t_cumw = torch.tensor(cumw if len(cumw) else np.zeros(1, np.float32), device=dev)
    t_starts = torch.tensor(starts, device=dev)
    walks = torch.empty((len(starts), walk_length), dtype=torch.int32, device=dev)
    _lib.check(lib.hicgat_n2v_walks(P(t_rowptr), P(t_col), P(t_cumw), n, P(t_starts), len(starts), walk_length,
                                    float(p), float(q), int(seed) & (2 ** 64 - 1), P(walks), _lib.stream(dev)),
               "hicgat_n2v_walks")
    return walks


def vocab_tables(counts, sample=1e-3, ns_exponent=0.75):
    """gensim 4 ``prepare_vocab`` keep probabilities and ``make_cum_table`` (domain 2^31 - 1)."""
    counts = np.asarray(counts, dtype=np.float64)
    thr = sample * counts.sum()
    with np.errstate(divide="ignore", invalid="ignore"):
        keep = np.where(counts > 0, np.minimum((np.sqrt(counts / thr) + 1.0) * (thr / counts), 1.0), 0.0)
    pw = counts ** ns_exponent
    cum = np.round(np.cumsum(pw) / pw.sum() * (2 ** 31 - 1)).astype(np.uint32)
    return keep.astype(np.float32), cum


def initial_vectors(walks, n_words, dimensions, w2v_seed=1):
    """gensim 4's initial input vectors: ``prep_vectors`` draws ``default_rng(seed).random((V, D))``
    mapped to U(-1/D, 1/D) for the vocabulary in its order, so node n gets row rank(n).  The order:
    ``prepare_vocab`` adds the words in first-appearance order of the corpus scan (the raw vocabulary
    dict), then ``sort_by_descending_frequency`` permutes them by ``np.argsort(count)[::-1]`` --
    numpy's default (unstable) sort, reversed, so tied words are NOT in first-appearance order; the
    same expression is applied here to the same count array.  The reference's
    ``.fit(window=25, min_count=1, batch_words=4)`` passes no seed, so Word2Vec's default seed 1
    applies.  (gensim is absent here: the rule is restated from its published source, unpinned.)"""
    flat = walks.reshape(-1)
    flat = flat[flat >= 0].cpu().numpy().astype(np.int64)
    counts = np.bincount(flat, minlength=n_words)
    words, first = np.unique(flat, return_index=True)
    scan = words[np.argsort(first)]                             # first-appearance order
    order = scan[np.argsort(counts[scan])[::-1]]                # gensim 4 sort_by_descending_frequency
    init = np.random.default_rng(seed=w2v_seed).random((len(order), dimensions), dtype=np.float32)
    init *= 2.0
    init -= 1.0
    init /= dimensions
    vec = np.zeros((n_words, dimensions), dtype=np.float32)     # a node no walk visits stays 0 (not in the vocab)
    vec[order] = init
    return vec


SMALL_VOCAB = 1024


def skipgram(walks, n_words, dimensions=512, window=25, epochs=5, negative=5, alpha=0.025, min_alpha=1e-4,
             sample=1e-3, seed=42, max_waves=None, w2v_seed=1):
    """Word2Vec(sg=1, hs=0) over the walks: returns the input vectors syn0 [n_words, dimensions].
    ``max_waves`` bounds the walks trained concurrently: on a Hi-C-sized vocabulary (58 loci for
    chr19 1 mb) concurrent Hogwild writers to the same rows would lose updates, so vocabularies
    below ``SMALL_VOCAB`` words train near-sequentially (n_words // 64 walks at once); larger ones
    keep n_words // 4 walks in flight (at most 4096)."""
    lib = _lib.lib()
    dev = walks.device
    nwalks, L = walks.shape
    counts = torch.bincount(walks[walks >= 0].long(), minlength=n_words).cpu().numpy()
    keep, cum = vocab_tables(counts, sample)
    t_keep = torch.tensor(keep, device=dev)
    t_cum = torch.tensor(cum.view(np.int32), device=dev)          # uint32 bits
    syn0 = torch.tensor(initial_vectors(walks, n_words, dimensions, w2v_seed), device=dev)
    syn1 = torch.zeros_like(syn0)
    st = _lib.stream(dev)
    if max_waves is None:
        # at most one concurrent walk per 64 words: sequential, like the reference's workers=1, for
        # a Hi-C chromosome at 1 mb / 500 kb (58 / 114 loci); measured on chr19 1 mb, 1 vs 14
        # concurrent walks give the same embedding structure (common-component share 0.984 vs
        # 0.980, profiles/r03b_n2v_study.json) at 20 vs 5 s
        max_waves = max(1, n_words // 64) if n_words < SMALL_VOCAB else max(1, min(4096, n_words // 4))
    for ep in range(epochs):
        _lib.check(lib.hicgat_n2v_sgns_epoch(P(walks), nwalks, L, P(t_keep), P(t_cum), n_words, dimensions, window,
                                             negative, float(alpha), float(min_alpha), ep, epochs,
                                             int(seed) & (2 ** 64 - 1), int(max_waves), P(syn0), P(syn1), st),
                   "hicgat_n2v_sgns_epoch")
    return syn0


def node2vec(matrix, dimensions=512, walk_length=150, num_walks=50, p=1.75, q=0.4, window=25, epochs=5,
             negative=5, alpha=0.025, min_alpha=1e-4, sample=1e-3, seed=42, device="cuda", max_waves=None):
    """[N, dimensions] node2vec embeddings of ``matrix`` (node order), HiC_GAT_generalize_directly.py's
    defaults."""
    walks = random_walks(matrix, num_walks, walk_length, p, q, seed, device)
    return skipgram(walks, np.asarray(matrix).shape[0], dimensions, window, epochs, negative, alpha, min_alpha,
                    sample, seed, max_waves=max_waves)


def embedding_stats(emb, truth=None):
    """Structure of an embedding matrix [N, F] (SURVEY 8(f) f4 has no reference vectors to compare):
    ``shared`` -- the share of the rows' energy in their common mean, ||mean||^2 / mean ||x_i||^2;
    ``cos_mean`` -- the mean pairwise cosine; ``locality`` -- Spearman of the pairwise distances
    of the CENTRED rows against the genomic separation |i - j| (positive: nearby loci embed nearby);
    ``truth_rho`` -- Spearman of those distances against ``truth`` (e.g. cont2dist of the contacts)."""
    from scipy.stats import spearmanr
    e = np.asarray(emb, dtype=np.float64)
    n = e.shape[0]
    mu = e.mean(0)
    shared = float(mu @ mu / np.mean(np.sum(e * e, 1)))
    u = e / np.maximum(np.linalg.norm(e, axis=1, keepdims=True), 1e-30)
    iu = np.triu_indices(n, 1)
    cos = (u @ u.T)[iu]
    c = e - mu
    d = np.sqrt(np.maximum(np.sum(c * c, 1)[:, None] + np.sum(c * c, 1)[None, :] - 2 * c @ c.T, 0))[iu]
    sep = (iu[1] - iu[0]).astype(np.float64)
    out = {"shared": shared, "cos_mean": float(cos.mean()), "cos_min": float(cos.min()),
           "norm_mean": float(np.linalg.norm(e, axis=1).mean()), "locality": float(spearmanr(d, sep)[0])}
    if truth is not None:
        out["truth_rho"] = float(spearmanr(d, np.asarray(truth, dtype=np.float64)[iu])[0])
    return out
