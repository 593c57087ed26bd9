"""The HiC-GNN_main.py training loop on the HIP path (a14), plus a CLI mirroring its flags
(list -> convert_to_matrix -> KRnorm on the GPU -> load_input -> train per conversion -> dSCC).

Loop semantics kept from HiC-GNN_main.py:117-132:
  Adam(lr) over model.parameters(); oldloss, lossdiff = 1, 1; truth = cont2dist(y, 0.5);
  while lossdiff > thresh: zero_grad; loss = MSE(model(x, ei), truth); lossdiff = |old - loss|;
  backward; step; old = loss.
The step runs the fused distance/loss kernel (the N x N matrix is never stored) and FlatAdam; the
loss comparison is the one device->host sync per step, as in the reference.  ``steps=K`` runs a
fixed number of steps instead (the deterministic parity protocol of SURVEY.md section 8(d)).
``loss="combined"`` is the HiC_GAT_generalize_directly.py:206-239 objective (MSE + alpha*(1-r)).
"""
import argparse
import ast
import sys

import numpy as np
import torch

from . import graph, metrics, ops
from .gat_models import MODELS
from .optim import FlatAdam


def train_step(model, opt, x, edge_index, truth, kind="mse", stats=None):
    """One step without any host sync: returns (loss tensor, stats tensor, coords)."""
    model.train()
    opt.zero_grad()
    loss, stats, coords = model.loss(x, edge_index, truth, kind, stats=stats)
    with ops.overlapped_param_grads(None if x.is_cuda else False):   # dW, db beside the backward
        loss.backward()
    opt.step()
    return loss, stats, coords


def train(model, data, truth, lr=1e-3, thresh=1e-8, steps=None, loss="mse", max_steps=1_000_000,
          on_step=None):
    """Returns (optimizer, per-step loss list).  ``truth`` is a ``graph.Truth``."""
    opt = FlatAdam(model.flat_parameters(), lr=lr)
    old, diff, hist = 1.0, 1.0, []
    stats = torch.empty(12, dtype=torch.float64, device=data.x.device)
    while (diff > thresh if steps is None else len(hist) < steps) and len(hist) < max_steps:
        model.train()
        opt.zero_grad()
        val, stats, _ = model.loss(data.x, data.edge_index, truth, loss, stats=stats)
        lv = float(val.item())
        diff = abs(old - lv)
        val.backward()
        opt.step()
        old = lv
        hist.append(lv)
        if on_step is not None:
            on_step(len(hist), lv)
    return opt, hist


def main(argv=None):
    p = argparse.ArgumentParser(description="Train a GAT-HiC model on the MI355X path "
                                            "(HiC-GNN_main.py flags).")
    p.add_argument("matrix", help="Hi-C list (bin_i bin_j count) or dense matrix text file")
    p.add_argument("features", help="N x F embedding text file (np.loadtxt), or 'node2vec' to generate the "
                                    "embeddings on the GPU from the contact matrix (hicgat.embed, the "
                                    "HiC_GAT_generalize_directly.py:150-155 call)")
    p.add_argument("-c", "--conversions", default="[.5]", help="conversion factor list, '[a, step, b]' or '[f]'")
    p.add_argument("-lr", "--learningrate", type=float, default=1e-3)
    p.add_argument("-th", "--threshold", type=float, default=1e-8)
    p.add_argument("--steps", type=int, default=None, help="fixed step count instead of the threshold rule")
    p.add_argument("--model", default="GATNetSelectiveResidualsUpdated", choices=sorted(MODELS))
    p.add_argument("--loss", default="mse", choices=["mse", "combined"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--out", default=None, help="prefix for <out>_weights.pt / _structure.pdb / _log.txt")
    p.add_argument("--no-kr", action="store_true", help="the input is already KR-normalised (skip KRnorm)")
    a = p.parse_args(argv)
    conv = ast.literal_eval(a.conversions)
    conv = list(np.arange(conv[0], conv[2], conv[1])) if len(conv) == 3 else [conv[0]]
    mat = np.loadtxt(a.matrix)
    if mat.shape[1] == 3:                       # HiC-GNN_main.py:75-78
        mat = graph.convert_to_matrix(mat)
    if a.features == "node2vec":                # node2vec on the raw contact graph (:150-155)
        from .embed import node2vec
        feats = node2vec(mat, seed=a.seed if a.seed else 42).cpu().numpy()
    else:
        feats = np.loadtxt(a.features).astype(np.float32)
    np.fill_diagonal(mat, 0)                    # :80
    if not a.no_kr:                             # :85-89 (Rscript normalize.R -> r_utils.R KRnorm)
        from .kr import KRnorm
        normed, keep = KRnorm(mat)
        mat = normed.cpu().numpy()
        feats = feats[keep.cpu().numpy()] if len(keep) != len(feats) else feats
    data = graph.load_input(mat, feats)
    best = None
    for f in conv:
        torch.manual_seed(a.seed)
        model = MODELS[a.model]().to(data.x.device)
        truth = graph.Truth.from_contacts(data.y, f)
        _, hist = train(model, data, truth, a.learningrate, a.threshold, a.steps, a.loss)
        coords = model.get_model(data.x.float(), data.edge_index).detach()
        rho = metrics.dscc(coords, truth.dense())
        print(f"conversion {f}: steps {len(hist)} loss {hist[-1]:.6g} dSCC {rho:.6f}")
        if best is None or rho > best[0]:
            best = (rho, f, hist[-1], model, coords)
    rho, f, l, model, coords = best
    print(f"Optimal conversion factor: {f}\nOptimal dSCC: {rho}")
    if a.out:
        from .io import write_pdb
        with open(f"{a.out}_log.txt", "w") as fh:
            fh.writelines([f"Optimal conversion factor: {f}\n", f"Optimal dSCC: {rho}\n", f"Final MSE loss: {l}\n"])
        torch.save(model.state_dict(), f"{a.out}_weights.pt")
        write_pdb(coords.cpu().numpy() * 100, f"{a.out}_structure.pdb")
    return 0


if __name__ == "__main__":
    sys.exit(main())
