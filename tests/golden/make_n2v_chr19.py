"""Generate ``n2v_chr19_1mb.npz``: the 512-d node2vec embedding of GM12878 chr19 1 mb made by this
repo's GPU node2vec (hicgat.embed.node2vec: walks + skip-gram in libhicgat.so) with the reference's
parameters (HiC_GAT_generalize_directly.py:150-155: dimensions=512, walk_length=150, num_walks=50,
p=1.75, q=0.4, window=25, seed=42), on the zero-diagonal contact matrix of the committed fixture
graph_chr19_1mb.npz -- the matrix HiC-GNN_main.py feeds the pipeline (:80, list -> matrix -> zero
diagonal).  BASELINE configs[0] names "512-d node2vec" features; node2vec / gensim are absent here,
so the same embedding file is then fed to BOTH sides: the CPU oracle (make_dscc_band.py --features
n2v) and the device pipeline (tests/test_gpu_parity.py::test_dscc_chr19_1mb_node2vec_matches_oracle).

Needs the GPU:  python tests/golden/make_n2v_chr19.py [out.npz [seed]]
(seed 43: ``n2v_chr19_1mb_s43.npz``, the second seed of the collapse check)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "..", "hic-gnn_amd")]


def main():
    from hicgat.embed import node2vec
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "n2v_chr19_1mb.npz")
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 42
    with np.load(os.path.join(HERE, "graph_chr19_1mb.npz"), allow_pickle=False) as z:
        a = np.array(z["matrix"], dtype=np.float64)
    np.fill_diagonal(a, 0)
    x = node2vec(a, seed=seed).cpu().numpy().astype(np.float32)
    assert x.shape == (a.shape[0], 512) and np.isfinite(x).all()
    np.savez(out, x=x, seed=np.int64(seed))
    print(f"node2vec chr19 1mb: {x.shape}, |x| mean {np.abs(x).mean():.4f} -> {out}")


if __name__ == "__main__":
    main()
