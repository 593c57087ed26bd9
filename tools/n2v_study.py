"""node2vec features for BASELINE configs[0] (GM12878 chr19 1 mb): embedding structure and the
flagship's fixed-K dSCC per skip-gram concurrency (max_waves) and seed, on the GPU.

    python tools/n2v_study.py [out.json]

For each (seed, max_waves): the reference's node2vec parameters (HiC_GAT_generalize_directly.py:
150-155) on the zero-diagonal contact matrix, ``embed.embedding_stats`` (shared-component share,
mean cosine, locality), then the HiC-GNN_main.py pipeline (KR, load_input, cont2dist(y, 0.5),
seed-0 weights, K = 3000 fixed steps, get_model, dSCC) with those features.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hic-gnn_amd"))

import hicgat  # noqa: E402
from hicgat import embed  # noqa: E402


def pipeline_dscc(a, x, K=3000):
    normed, keep = hicgat.kr.KRnorm(a.copy())
    keep = keep.cpu().numpy()
    x = x[keep] if len(keep) != len(x) else x
    data = hicgat.load_input(normed.cpu().numpy(), x.astype(np.float32))
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().cuda()
    tr = hicgat.Truth.from_contacts(data.y, 0.5)
    _, hist = hicgat.train.train(model, data, tr, steps=K)
    with torch.no_grad():
        coords = model.get_model(data.x.float(), data.edge_index)
    return float(hicgat.metrics.dscc(coords, tr.dense())), float(hist[-1]), tr.dense().double().cpu().numpy()


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    g = np.load(os.path.join(ROOT, "tests", "golden", "graph_chr19_1mb.npz"))
    a = np.array(g["matrix"], dtype=np.float64)
    np.fill_diagonal(a, 0)
    rows = []
    for seed in (42, 43):
        for mw in (1, 4, 14, 64):
            t0 = time.time()
            e = embed.node2vec(a, seed=seed, max_waves=mw).cpu().numpy()
            torch.cuda.synchronize()
            t_emb = time.time() - t0
            rho, loss, truth = pipeline_dscc(a, e)
            st = embed.embedding_stats(e, truth)
            row = dict(seed=seed, max_waves=mw, seconds=t_emb, dscc_k3000=rho, final_loss=loss, **st)
            rows.append(row)
            print(json.dumps(row), flush=True)
    # the fixture's random features (0.1 N(0,1)) for comparison
    x = np.load(os.path.join(ROOT, "tests", "golden", "model_GATNetSelectiveResidualsUpdated.npz"))["x"]
    rho, loss, truth = pipeline_dscc(a, np.asarray(x))
    row = dict(features="fixture 0.1*N(0,1)", dscc_k3000=rho, final_loss=loss, **embed.embedding_stats(x, truth))
    rows.append(row)
    print(json.dumps(row), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
