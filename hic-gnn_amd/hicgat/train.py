"""The HiC-GNN_main.py training loop on the HIP path (a14), plus a CLI mirroring its flags
(list -> convert_to_matrix -> KRnorm on the GPU -> load_input -> train per conversion -> dSCC).

Loop semantics kept from HiC-GNN_main.py:117-132:
  Adam(lr) over model.parameters(); oldloss, lossdiff = 1, 1; truth = cont2dist(y, 0.5);
  while lossdiff > thresh: zero_grad; loss = MSE(model(x, ei), truth); lossdiff = |old - loss|;
  backward; step; old = loss.
The step runs the fused distance/loss kernel (the N x N matrix is never stored) and FlatAdam; the
loss comparison is the one device->host sync per step, as in the reference.  ``steps=K`` runs a
fixed number of steps instead (the deterministic parity protocol of SURVEY.md section 8(d)).
``loss="combined"`` is the HiC_GAT_generalize_directly.py:206-239 objective (MSE + alpha*(1-r));
``loss="contrastive"`` the train_and_test_same_res_GAT_node2vec.py:98-134 one (0.1 * mean_{i<j}
|T - D|, float64 as the reference's float64 truth makes it: the lossdiff rule reads that fp64 value).
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
    pk = ops.step_pack(model, x) if x.is_cuda else None   # the tail's packed weights ride in the first launch
    if pk is not None:
        opt.zero_grad(pack=pk)
    else:
        opt.zero_grad()
    with ops.prepacked(model, pk):
        loss, stats, coords = model.loss(x, edge_index, truth, kind, stats=stats)
    with ops.overlapped_param_grads(None if x.is_cuda else False):   # dW, db beside the backward
        ops.backward_from_loss(loss)
    opt.step()
    return loss, stats, coords


GRAPH_WARMUP = 2   # eager steps before the step is captured (real training steps, in the history)


def train(model, data, truth, lr=1e-3, thresh=1e-8, steps=None, loss="mse", max_steps=1_000_000,
          on_step=None, graph=None, dscc_history=None, print_interval=0):
    """Returns (optimizer, per-step loss list).  ``truth`` is a ``graph.Truth``.

    ``graph`` (default: on for device tensors): after ``GRAPH_WARMUP`` eager steps the step is
    captured once (``graphs.CapturedStep``) and replayed; the loss is still read on the host every
    step for the ``lossdiff`` rule (HiC-GNN_main.py:128) -- replays give the same bits as eager steps.
    ``dscc_history`` (a list): the dSCC of every step's forward coordinates against the target, as
    HiC_GAT_generalize_directly.py:242-247 appends it; ``print_interval`` > 0 prints its progress line
    (:256) every that many steps."""
    from .graphs import CapturedStep
    opt = FlatAdam(model.flat_parameters(), lr=lr)
    use_graph = data.x.is_cuda if graph is None else bool(graph)
    if use_graph:
        opt.enable_device_step()
    old, diff, hist = 1.0, 1.0, []
    stats = torch.empty(12, dtype=torch.float64, device=data.x.device)
    score = truth.scoring() if dscc_history is not None else None

    def step():
        return train_step(model, opt, data.x, data.edge_index, truth, loss, stats)

    replay = None
    while (diff > thresh if steps is None else len(hist) < steps) and len(hist) < max_steps:
        if use_graph and replay is None and len(hist) >= GRAPH_WARMUP:
            replay = CapturedStep(step, warmup=0)     # captured, not run: the replay below is this step
        val, st, coords = replay() if replay is not None else step()
        # the one device -> host read per step (the contrastive total is float64 in the reference)
        lv = float(st[10].item()) if loss == "contrastive" else float(val.item())
        diff = abs(old - lv)
        old = lv
        hist.append(lv)
        if score is not None:
            dscc_history.append(metrics.dscc(coords, score))
            if print_interval and (len(hist) - 1) % print_interval == 0:
                print(f"Iteration [{len(hist) - 1}], Total Loss: {float(stats[7]):.6g}, dSCC: {dscc_history[-1]}, "
                      f"Loss Diff: {diff}")
        if on_step is not None:
            on_step(len(hist), lv)
    opt.sync_step_count()     # replays advanced only the device count
    return opt, hist


def cpu_state_dict(model):
    """The state_dict as plain CPU tensors (no views into FlatAdam's device buffers), so the saved
    .pt loads with a bare ``torch.load(path)`` on a CPU-only host, as the reference's evaluate /
    generalise scripts do (evaluate.py:87, HiC_GAT_generalize_directly.py:313)."""
    return {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}


def parse_conversions(text):
    """HiC-GNN_main.py:51-58: '[a, step, b]' -> np.arange(a, b, step), '[f]' -> [f]."""
    conv = ast.literal_eval(text)
    if len(conv) == 3:
        return list(np.arange(conv[0], conv[2], conv[1]))
    if len(conv) == 1:
        return [conv[0]]
    raise ValueError("Invalid conversion input.")


def main(argv=None):
    """HiC-GNN_main.py's pipeline: list -> convert_to_matrix -> zero diagonal -> KRnorm ->
    embeddings -> load_input -> one model per conversion value -> best dSCC -> weights / PDB / log.

    As in the reference (HiC-GNN_main.py:108-132), EVERY conversion value trains a fresh model
    against ``cont2dist(y, 0.5)`` and is scored against that same truth: the value only labels the
    run (the reference never passes it to cont2dist); the models differ by their random init (one
    seed for the whole sweep, the RNG stream continuing from model to model)."""
    p = argparse.ArgumentParser(description="Train a GAT-HiC model on the MI355X path "
                                            "(HiC-GNN_main.py flags).")
    p.add_argument("matrix", help="Hi-C list (bin_i bin_j count) or dense matrix text file")
    p.add_argument("features", help="N x F embedding text file (np.loadtxt), or 'node2vec' to generate the "
                                    "embeddings on the GPU from the zero-diagonal contact matrix (hicgat.embed, "
                                    "the HiC_GAT_generalize_directly.py:150-155 call)")
    p.add_argument("-c", "--conversions", default="[.1,.1,2]", help="conversion list, '[a, step, b]' or '[f]' "
                                                                    "(HiC-GNN_main.py:33)")
    p.add_argument("-lr", "--learningrate", type=float, default=1e-3)
    p.add_argument("-th", "--threshold", type=float, default=1e-8)
    p.add_argument("--steps", type=int, default=None, help="fixed step count instead of the threshold rule")
    p.add_argument("--model", default="GATNetSelectiveResidualsUpdated", choices=sorted(MODELS))
    p.add_argument("--loss", default="mse", choices=["mse", "combined", "contrastive"])
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--out", default=None, help="prefix for <out>_weights.pt / _structure.pdb / _log.txt")
    p.add_argument("--no-kr", action="store_true", help="the input is already KR-normalised (skip KRnorm)")
    a = p.parse_args(argv)
    conv = parse_conversions(a.conversions)
    mat = np.loadtxt(a.matrix)
    if mat.shape[1] == 3:                       # HiC-GNN_main.py:75-78
        print("Converting coordinate list format to matrix.")
        mat = graph.convert_to_matrix(mat)
    np.fill_diagonal(mat, 0)                    # :80
    if a.features == "node2vec":                # node2vec on the zero-diagonal contact graph (:150-155)
        from .embed import node2vec
        feats = node2vec(mat, seed=a.seed if a.seed else 42).cpu().numpy()
    else:
        feats = np.loadtxt(a.features).astype(np.float32)
    if not a.no_kr:                             # :85-89 (Rscript normalize.R -> r_utils.R KRnorm)
        from .kr import KRnorm
        normed, keep = KRnorm(mat)
        mat = normed.cpu().numpy()
        feats = feats[keep.cpu().numpy()] if len(keep) != len(feats) else feats
    data = graph.load_input(mat, feats)
    truth = graph.Truth.from_contacts(data.y, 0.5)     # :120, the same for every conversion
    torch.manual_seed(a.seed)
    runs = []
    for f in conv:
        print(f"Training model using conversion value {f}.")
        model = MODELS[a.model]().to(data.x.device)
        _, hist = train(model, data, truth, a.learningrate, a.threshold, a.steps, a.loss)
        coords = model.get_model(data.x.float(), data.edge_index).detach()
        rho = metrics.dscc(coords, truth.scoring())
        print(f"conversion {f}: steps {len(hist)} loss {hist[-1]:.6g} dSCC {rho:.6f}")
        runs.append((rho, f, hist[-1], model, coords))
    k = [r[0] for r in runs].index(max(r[0] for r in runs))     # first maximum, as list.index(max)
    rho, f, loss, model, coords = runs[k]
    print(f"Optimal conversion factor: {f}")
    print(f"Optimal dSCC: {rho}")
    if a.out:
        from .io import write_pdb
        with open(f"{a.out}_log.txt", "w") as fh:        # :155-156
            fh.writelines([f"Optimal conversion factor: {f}\n", f"Optimal dSCC: {rho}\n", f"Final MSE loss: {loss}\n"])
        torch.save(cpu_state_dict(model), f"{a.out}_weights.pt")
        write_pdb(coords.cpu().numpy() * 100, f"{a.out}_structure.pdb")
        print(f"Saved trained model to {a.out}_weights.pt")
        print(f"Saved optimal structure to {a.out}_structure.pdb")
    return 0


if __name__ == "__main__":
    sys.exit(main())
