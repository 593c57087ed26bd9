"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own code -- with one
qualification: the GAT arithmetic in them is NOT the reference's (parity unpinned, see below).

Run in the build container only (the reference tree does not exist on the GPU box):

    python tests/golden/make_golden.py /root/reference [align]   # "align": only the align_* fixtures

It imports the reference ``utils.py`` / ``models.py`` (``/root/reference``) with the stand-ins in
``tests/golden/_stubs`` for the absent ``torch_geometric`` / ``torch_sparse`` packages and records:

* ``graph_<case>.npz``  -- ``utils.convert_to_matrix`` (utils.py:10-26), ``utils.load_input``
  (utils.py:29-73: networkx edge list, masked self loops, symmetric CSR) and ``utils.cont2dist``
  (utils.py:75-80) at factors 0.5 and 1.0, for GM12878 chr19 1mb / 500kb (``Data/*.txt``) and a
  synthetic 3-column list with duplicates, gaps and asymmetric entries.
* ``model_<name>.npz``  -- a reference model class (``models.py:614-691`` / ``:1010-1047``) built
  under ``torch.manual_seed(0)`` on chr19 1mb with 0.1*N(0,1) features: initial state_dict,
  forward distance matrix, coordinates, MSE vs cont2dist(y, 0.5), every parameter gradient, and the
  combined-loss value of ``HiC_GAT_generalize_directly.py:206-225``.
* ``model_Net.npz``    -- the baseline SAGE model (models.py:14-55 over layers.py:12-79) on chr19
  1mb: init state, SAGE aggregate, distances, coordinates, MSE, gradients; plus the key/shape
  layout of the shipped ``Outputs/GM12878_1mb_chr19_list_weights.pt`` (safe loader).
* ``align_chr19_f<F>.npz`` -- ``utils.domain_alignment`` (utils.py:83-109) on the chr19 1 mb /
  500 kb lists with seeded float32 embeddings of width F (512: rank-deficient Procrustes, 32: full
  rank).
* ``train_<name>.npz``  -- the ``HiC-GNN_main.py:117-132`` loop run for a fixed K on the same input
  (deterministic algorithms), loss history and final coordinates.

What is pinned by the reference and what is not:

* pinned (reference code ran): convert_to_matrix, load_input's edge construction and cont2dist
  (``graph_*``), domain_alignment (``align_*``), the SAGE baseline ``Net`` (its SAGEConv is the
  reference's own ``layers.py``), and the COMPOSITION of the GAT models -- the tail Linear /
  LayerNorm / residual wiring, parameter registration order and init, cdist, MSE, the combined
  loss and the training loop of ``models.py`` / ``HiC-GNN_main.py``;
* NOT pinned: the GATConv values inside ``model_GAT*.npz`` / ``train_GAT*.npz``.  PyG 1.7.2 is
  absent, so ``models.py``'s ``GATConv`` resolves to the stand-in
  ``_stubs/torch_geometric/nn.py``, which IS ``oracle.gat.GATConv`` (the restatement of PyG
  1.7.2's published code path), and the CSR the models see comes through the ``_stubs/torch_sparse``
  stand-in.  Those fixtures therefore check the oracle's GAT arithmetic against itself: the GAT
  kernels' parity is "parity unpinned" (DESIGN.md section 4).

Only data is written (inputs and expected outputs); no reference source is copied.
"""
import os
import sys

import numpy as np
import torch
from scipy.stats import pearsonr

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _import_reference(ref):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(HERE, "_stubs"))
    sys.path.insert(0, ref)
    import models as ref_models  # noqa: E402  (reference models.py)
    import utils as ref_utils    # noqa: E402  (reference utils.py)
    return ref_utils, ref_models


def graph_case(ref_utils, name, lst):
    mat = ref_utils.convert_to_matrix(lst)
    n = mat.shape[0]
    rng = np.random.default_rng(1)
    feats = (0.1 * rng.standard_normal((n, 512))).astype(np.float32)
    data = ref_utils.load_input(mat.copy(), feats)
    st = data.edge_index.storage
    out = dict(
        list=lst, matrix=mat,
        rowptr=st.rowptr().numpy(), col=st.col().numpy(), value=st.value().numpy(),
        y=data.y.numpy(),
        truth05=ref_utils.cont2dist(data.y.clone(), 0.5).numpy(),
        truth1=ref_utils.cont2dist(data.y.clone(), 1).numpy(),
    )
    np.savez_compressed(os.path.join(HERE, f"graph_{name}.npz"), **out)
    print(f"graph_{name}: N={n} nnz={len(out['col'])}")
    return mat, data


def synth_list(seed=7):
    """Ragged 3-column Hi-C list: gaps in the bin ids, repeated pairs, lower-triangle and
    asymmetric entries, an isolated bin whose row ends up all zero (and is removed)."""
    rng = np.random.default_rng(seed)
    bins = np.sort(rng.choice(np.arange(0, 400) * 50000, size=256, replace=False))
    rows = []
    for _ in range(3000):
        i, j = rng.integers(0, 256, size=2)
        if rng.random() < 0.8:
            i, j = min(i, j), max(i, j)
        rows.append((bins[i], bins[j], float(rng.integers(1, 500))))
    rows.append((bins[3], bins[3], 77.0))                 # a pure self contact
    rows.extend(rows[:40])                                 # repeats (last write wins)
    return np.array(rows, dtype=np.float64)


def model_case(ref_utils, ref_models, cls_name, data, seed=0):
    torch.manual_seed(seed)
    model = getattr(ref_models, cls_name)()
    x = data.x.float()
    truth = ref_utils.cont2dist(data.y.clone(), 0.5)
    state = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    model.zero_grad()
    out = model(x, data.edge_index)
    coords = model.get_model(x, data.edge_index)
    mse = torch.nn.MSELoss()(out.float(), truth.float())
    mse.backward()
    grads = {f"grad::{k}": p.grad.detach().numpy().copy() for k, p in model.named_parameters()}
    n = truth.shape[0]
    idx = torch.triu_indices(n, n, offset=1)
    r = pearsonr(truth[idx[0], idx[1]].numpy(), torch.cdist(coords, coords)[idx[0], idx[1]].detach().numpy())[0]
    alpha = min(1.0, 0.1 + (1.0 / (mse.item() + 1e-6)))
    total = mse.item() + alpha * (1 - r)
    np.savez_compressed(
        os.path.join(HERE, f"model_{cls_name}.npz"),
        x=x.numpy(), truth=truth.float().numpy(), out=out.detach().numpy(), coords=coords.detach().numpy(),
        mse=np.float64(mse.item()), pearson=np.float64(r), alpha=np.float64(alpha), total=np.float64(total),
        **{f"state::{k}": v for k, v in state.items()}, **grads)
    print(f"model_{cls_name}: mse={mse.item():.8g} r={r:.8g}")
    return model


def net_case(ref_utils, ref_models, ref, mat, seed=0):
    """The baseline ``Net`` (models.py:14-55, SAGEConv of layers.py:12-79) on chr19 1mb.

    Features are 1.5*N(0,1) so that ``x.long()`` (layers.py:64) keeps non-zero integers.  The
    key/shape layout of the shipped trained state_dict (``Outputs/*_weights.pt``, read with
    ``weights_only=True``) is recorded too."""
    rng = np.random.default_rng(5)
    feats = (1.5 * rng.standard_normal((mat.shape[0], 512))).astype(np.float32)
    data = ref_utils.load_input(mat.copy(), feats)
    torch.manual_seed(seed)
    model = ref_models.Net()
    x = data.x.float()
    truth = ref_utils.cont2dist(data.y.clone(), 0.5)
    state = {k: v.detach().clone().numpy() for k, v in model.state_dict().items()}
    out = model(x, data.edge_index)
    coords = model.get_model(x, data.edge_index)
    agg = model.conv.message_and_aggregate(data.edge_index, (x, x))
    mse = torch.nn.MSELoss()(out.float(), truth.float())
    mse.backward()
    grads = {f"grad::{k}": p.grad.detach().numpy().copy() for k, p in model.named_parameters()}
    trained = torch.load(os.path.join(ref, "Outputs", "GM12878_1mb_chr19_list_weights.pt"), weights_only=True,
                         map_location="cpu")
    np.savez_compressed(
        os.path.join(HERE, "model_Net.npz"),
        x=x.numpy(), agg=agg.detach().numpy(), out=out.detach().numpy(), coords=coords.detach().numpy(),
        mse=np.float64(mse.item()), trained_keys=np.array(list(trained.keys())),
        trained_shapes=np.array([list(v.shape) + [0] * (2 - v.dim()) for v in trained.values()]),
        **{f"state::{k}": v for k, v in state.items()}, **grads)
    print(f"model_Net: mse={mse.item():.8g}; trained keys {list(trained.keys())}")


def train_case(ref_utils, ref_models, cls_name, data, steps=25, seed=0):
    torch.use_deterministic_algorithms(True)
    torch.manual_seed(seed)
    model = getattr(ref_models, cls_name)()
    x = data.x.float()
    truth = ref_utils.cont2dist(data.y.clone(), 0.5)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    crit = torch.nn.MSELoss()
    hist = []
    oldloss = 1
    for _ in range(steps):                    # HiC-GNN_main.py:123-132 with a fixed K
        model.train()
        opt.zero_grad()
        out = model(x, data.edge_index)
        loss = crit(out.float(), truth.float())
        _ = abs(oldloss - loss)
        loss.backward()
        opt.step()
        oldloss = loss
        hist.append(loss.item())
    coords = model.get_model(x, data.edge_index).detach().numpy()
    np.savez_compressed(os.path.join(HERE, f"train_{cls_name}.npz"), loss=np.array(hist),
                        coords=coords, steps=np.int64(steps))
    print(f"train_{cls_name}: loss {hist[0]:.6g} -> {hist[-1]:.6g}")


def align_case(ref_utils, l1, l5, f=512, seed=11):
    """utils.domain_alignment (utils.py:83-109) on the chr19 1 mb / 500 kb lists with seeded float32
    embeddings (node2vec's dtype): the fitted 500 kb embeddings the reference produces."""
    n1 = len(np.unique(np.concatenate([l1[:, 0], l1[:, 1]])))
    n5 = len(np.unique(np.concatenate([l5[:, 0], l5[:, 1]])))
    rng = np.random.default_rng(seed)
    e1 = rng.standard_normal((n1, f)).astype(np.float32)
    e5 = rng.standard_normal((n5, f)).astype(np.float32)
    fit = ref_utils.domain_alignment(l1, l5, e1, e5)
    np.savez_compressed(os.path.join(HERE, f"align_chr19_f{f}.npz"), list1=l1, list2=l5, emb1=e1, emb2=e5,
                        fitembed=fit)
    print(f"align_chr19_f{f}: {e1.shape} {e5.shape} -> {fit.shape} {fit.dtype}")


def main(ref, only=None):
    torch.set_num_threads(1)
    ref_utils, ref_models = _import_reference(ref)
    l1 = np.loadtxt(os.path.join(ref, "Data", "GM12878_1mb_chr19_list.txt"))
    l5 = np.loadtxt(os.path.join(ref, "Data", "GM12878_500kb_chr19_list.txt"))
    if only in (None, "align"):
        align_case(ref_utils, l1, l5, 512)
        align_case(ref_utils, l1, l5, 32)
    if only is not None:
        return
    _, data1 = graph_case(ref_utils, "chr19_1mb", l1)
    graph_case(ref_utils, "chr19_500kb", l5)
    graph_case(ref_utils, "synth256", synth_list())
    for cls in ("GATNetSelectiveResidualsUpdated", "GATNetHeadsChanged3LayersLeakyReLUv2"):
        model_case(ref_utils, ref_models, cls, data1)
    train_case(ref_utils, ref_models, "GATNetSelectiveResidualsUpdated", data1)
    net_case(ref_utils, ref_models, ref, ref_utils.convert_to_matrix(l1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference", sys.argv[2] if len(sys.argv) > 2 else None)
