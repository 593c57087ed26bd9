"""Cross-resolution generalisation on the GPU.

* ``domain_alignment(list1, list2, embeddings1, embeddings2)`` -- ``utils.py:83-109``: the bins of
  the two resolutions that line up are matched from the two contact lists (integer host logic on
  the lists, as in the reference), then the orthogonal Procrustes rotation R = U V^T of
  svd(A^T B) maps ``embeddings2`` onto ``embeddings1``'s frame: A^T B and embeddings2 @ R run on
  the fp32 MFMA GEMM of libhicgat.so, the 512 x 512 SVD on the device solver (torch.linalg.svd).
* ``generalize(...)`` -- ``HiC_GAT_generalize_directly.py:312-336``: the trained model applied to
  the aligned embeddings of the untrained resolution, scored by dSCC against
  cont2dist(normed_untrained, conversion).
* ``main()`` -- the driver's CLI (list_trained list_untrained, trains the 1 mb model with the
  combined loss and the threshold rule when no weights file exists, then generalises).

When A^T B is rank deficient (fewer matched bins than embedding dimensions) R is not unique on the
null space: any maximiser is a valid Procrustes solution, and which one a LAPACK build returns is
implementation detail (tests check orthogonality, the optimum and R on the range).
"""
import argparse
import os
import sys

import numpy as np
import torch

from . import graph, kernels, metrics


def matched_rows(list1, list2):
    """utils.py:84-104 -- rows of embeddings2 (A) and embeddings1 (B) whose bins line up."""
    list1 = np.asarray(list1)
    list2 = np.asarray(list2)
    idx1 = np.unique(list1[:, 0]).astype(int)
    diff1 = min(idx1[1:] - idx1[:-1])
    idx2 = np.unique(list2[:, 0]).astype(int)
    diff2 = min(idx2[1:] - idx2[:-1])
    bins = int(diff1 / (2 * diff2))
    a_rows, b_rows = [], []
    for i in range(bins + 1):
        a_rows.append(np.where(np.isin(idx2 + i * diff2, idx1))[0])
        b_rows.append(np.where(np.isin(idx1, idx2 + i * diff2))[0])
    return np.concatenate(a_rows), np.concatenate(b_rows)


def procrustes(A, B):
    """R = argmin ||A R - B||_F over orthogonal R (scipy.linalg.orthogonal_procrustes): U V^T of
    svd(A^T B).  A, B: [K, F] float32 device tensors; A^T B on the MFMA GEMM (K-split)."""
    K_ = kernels.default()
    F = A.shape[1]
    M = torch.empty((F, B.shape[1]), dtype=torch.float32, device=A.device)
    splits = max(1, min(A.shape[0] // 256, 64))
    K_.gemm(1, 1, F, B.shape[1], A.shape[0], A, B, M, splits=splits, name="gemm_procrustes")
    U, _, Vh = torch.linalg.svd(M.double(), full_matrices=False)
    return (U @ Vh).float()


def domain_alignment(list1, list2, embeddings1, embeddings2, device="cuda"):
    """utils.py:83-109 on the device -> embeddings2 @ R (float32, [N2, F])."""
    e1 = torch.as_tensor(np.asarray(embeddings1, dtype=np.float32)).to(device)
    e2 = torch.as_tensor(np.asarray(embeddings2, dtype=np.float32)).to(device)
    ia, ib = matched_rows(list1, list2)
    A = e2.index_select(0, torch.as_tensor(ia, device=device)).contiguous()
    B = e1.index_select(0, torch.as_tensor(ib, device=device)).contiguous()
    R = procrustes(A, B)
    out = torch.empty((e2.shape[0], R.shape[1]), dtype=torch.float32, device=device)
    # fitembed = embeddings2 @ R: C = A B with B row-major [K, N] (b_kmajor)
    kernels.default().gemm(0, 1, e2.shape[0], R.shape[1], e2.shape[1], e2, R, out, name="gemm_procrustes")
    return out


def generalize(model, list_trained, list_untrained, emb_trained, emb_untrained, normed_untrained, conversion=1,
               device="cuda"):
    """HiC_GAT_generalize_directly.py:312-336 -> (dSCC, coords [N2, 3])."""
    fit = domain_alignment(list_trained, list_untrained, emb_trained, emb_untrained, device)
    data = graph.load_input(np.array(normed_untrained, dtype=np.float64), fit, device=device)
    truth = graph.cont2dist(data.y, conversion).float()
    model.eval()
    with torch.no_grad():
        coords = model.get_model(data.x.float(), data.edge_index)
    return metrics.dscc(coords, truth), coords


def main(argv=None):
    from . import kr, train
    from .gat_models import MODELS
    from .io import write_pdb
    p = argparse.ArgumentParser(description="Generalise a trained GAT-HiC model to another resolution "
                                            "(HiC_GAT_generalize_directly.py flags).")
    p.add_argument("list_trained")
    p.add_argument("list_untrained")
    p.add_argument("embeddings_trained", help="N1 x F text file (np.loadtxt), or 'node2vec': generated on the GPU "
                                              "from the zero-diagonal contact matrix (:148-160)")
    p.add_argument("embeddings_untrained", help="N2 x F text file, or 'node2vec' (:162-173)")
    p.add_argument("--seed", type=int, default=42, help="node2vec seed (the reference's Node2Vec(seed=42))")
    p.add_argument("-lr", "--learningrate", type=float, default=0.001)
    p.add_argument("-thresh", "--loss_diff_threshold", type=float, default=1e-8)
    p.add_argument("--conversion", type=float, default=1.0)
    p.add_argument("--model", default="GATNetSelectiveResidualsUpdated", choices=sorted(MODELS))
    p.add_argument("--weights", default=None, help="trained state_dict (.pt); trained here when missing")
    p.add_argument("--steps", type=int, default=None)
    p.add_argument("--out", default=None, help="prefix for the weights / PDB / log files")
    p.add_argument("-print_interval", "--print_interval", type=int, default=10,
                   help="print MSE and dSCC every this many steps (:87)")
    a = p.parse_args(argv)
    l1, l2 = np.loadtxt(a.list_trained), np.loadtxt(a.list_untrained)
    normed, emb = [], []
    for lst, src in ((l1, a.embeddings_trained), (l2, a.embeddings_untrained)):
        m = graph.convert_to_matrix(lst)
        np.fill_diagonal(m, 0)                  # :113-126 (the saved *_matrix.txt)
        if src == "node2vec":                   # node2vec on that zero-diagonal matrix (:150-173)
            from .embed import node2vec
            emb.append(node2vec(m, seed=a.seed).cpu().numpy())
        else:
            emb.append(np.loadtxt(src))
        normed.append(kr.KRnorm(m)[0].cpu().numpy())
    e1, e2 = emb
    model = MODELS[a.model]().cuda()
    if a.weights and os.path.isfile(a.weights):
        model.load_state_dict(torch.load(a.weights, weights_only=True))
    else:
        data = graph.load_input(normed[0], e1.astype(np.float32))
        truth = graph.Truth.from_contacts(data.y, a.conversion)
        dscc_hist = []      # the per-step dSCC of :242-247 (the forward's coordinates before the update)
        _, hist = train.train(model, data, truth, a.learningrate, a.loss_diff_threshold, a.steps, "combined",
                              dscc_history=dscc_hist, print_interval=a.print_interval)
        print(f"trained {len(hist)} steps, final loss {hist[-1]:.6g}")
        print(f"\nOptimal dSCC after training: {dscc_hist[-1]}")                          # :273
        print(f"dSCC Loss - Mean: {np.mean(dscc_hist)}, Max: {np.max(dscc_hist)}")         # :278-280
        if a.weights:
            torch.save(train.cpu_state_dict(model), a.weights)
    rho, coords = generalize(model, l1, l2, e1, e2, normed[1], a.conversion)
    print(f"Optimal dSCC for generalized data: {rho}")
    if a.out:
        write_pdb(coords.cpu().numpy() * 100, f"{a.out}_generalized_structure.pdb")
        with open(f"{a.out}_generalized_log.txt", "w") as fh:
            fh.writelines([f"Optimal dSCC: {rho}\n"])
    return 0


if __name__ == "__main__":
    sys.exit(main())
