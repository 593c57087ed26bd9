"""Oracle: loss, training loop and dSCC of the GAT-HiC hot path (TEST INFRASTRUCTURE ONLY).

* ``mse_loss``            -- ``HiC-GNN_main.py:127``: ``MSELoss()(out.float(), truth.float())`` over
                             all N*N entries (diagonal included).
* ``combined_loss``       -- ``HiC_GAT_generalize_directly.py:206-225``: MSE + alpha*(1 - r), r the
                             float64 Pearson of the upper-triangle distances, *no gradient* through
                             r, alpha = min(1, 0.1 + 1/(mse + 1e-6)).
* ``contrastive_loss``    -- ``train_and_test_same_res_GAT_node2vec.py:107-134``: 0.1 * mean over the
                             upper triangle (offset 1) of |truth - cdist(coords)|, truth float64, so
                             the difference and the mean are float64; differentiable (no MSE term).
* ``train``               -- ``HiC-GNN_main.py:117-132`` loop (Adam lr 1e-3, |dloss| <= thresh stop),
                             with an optional fixed step count.
* ``dscc``                -- ``HiC-GNN_main.py:135-139``: Spearman of the triu distances.
"""
import numpy as np
import torch
from scipy.stats import pearsonr, spearmanr


def mse_loss(out, truth):
    return torch.nn.functional.mse_loss(out.float(), truth.float())


def pearson_r(coords, truth):
    """``HiC_GAT_generalize_directly.py:210-220``: float64 Pearson on the triu pairs, no grad."""
    n = truth.shape[0]
    idx = torch.triu_indices(n, n, offset=1)
    dist_truth = truth[idx[0], idx[1]].detach().numpy()
    dist_out = torch.cdist(coords, coords)[idx[0], idx[1]].detach().numpy()
    return float(pearsonr(dist_truth, dist_out)[0])


def combined_loss(out, coords, truth):
    """Returns ``(total, mse, r, alpha)``; grad(total) == grad(mse)."""
    mse = mse_loss(out, truth)
    r = pearson_r(coords, truth)
    alpha = min(1.0, 0.1 + (1.0 / (mse.item() + 1e-6)))
    return mse + alpha * (1 - r), mse, r, alpha


def contrastive_loss(coords, truth):
    """``train_and_test_same_res_GAT_node2vec.py:107-134``: ``idx = triu_indices(n, n, offset=1)``;
    ``dist_truth = truth[idx]`` (float64), ``dist_out = cdist(coords, coords)[idx]`` (float32);
    ``0.0 + 0.1 * mean(abs(dist_truth - dist_out))`` -- float64, its gradient cast back to float32 at
    ``dist_out``.  cdist in ``gat.CDIST_MODE`` (the reference's default mode; tests against the
    exact-distance kernels switch it, as for the MSE)."""
    from . import gat
    n = truth.shape[0]
    idx = torch.triu_indices(n, n, offset=1)
    dist_truth = truth[idx[0], idx[1]].to(torch.float64)
    dist_out = torch.cdist(coords, coords, p=2, compute_mode=gat.CDIST_MODE)[idx[0], idx[1]]
    return 0.0 + 0.1 * torch.mean(torch.abs(dist_truth - dist_out))


def dscc(coords, truth):
    """``HiC-GNN_main.py:135-139``: Spearman(truth triu, cdist(coords) triu)."""
    n = truth.shape[0]
    idx = torch.triu_indices(n, n, offset=1)
    dist_truth = truth[idx[0], idx[1]]
    dist_out = torch.cdist(coords, coords)[idx[0], idx[1]]
    return float(spearmanr(dist_truth.detach().numpy(), dist_out.detach().numpy())[0])


def train(model, x, adj, truth, lr=1e-3, thresh=1e-8, steps=None, loss="mse", max_steps=100000,
          on_step=None):
    """``HiC-GNN_main.py:117-132`` (``loss="mse"``) or ``HiC_GAT_generalize_directly.py:202-239``
    (``loss="combined"``).  With ``steps`` set, runs exactly that many steps (fixed-K protocol) and
    ignores ``thresh``.  Returns the list of per-step loss values (float)."""
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    old, diff, hist = 1.0, 1.0, []
    while (diff > thresh if steps is None else len(hist) < steps) and len(hist) < max_steps:
        model.train()
        opt.zero_grad()
        if loss == "mse":
            out = model(x, adj)
            val = mse_loss(out, truth)
        elif loss == "contrastive":
            val = contrastive_loss(model.get_model(x, adj), truth)
        else:
            coords = model.get_model(x, adj)
            out = torch.cdist(coords, coords, p=2)
            val, _, _, _ = combined_loss(out, coords, truth)
        lv = float(val.item())
        diff = abs(old - lv)
        val.backward()
        opt.step()
        old = lv
        hist.append(lv)
        if on_step is not None:
            on_step(len(hist), lv)
    return hist


def _fmaf(a, b, c):
    """float32 fused multiply-add, exact via float64 (a*b of two float32 is exact in float64)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def adam_reference_step(p, g, m, v, step, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8):
    """torch 2.x ``_single_tensor_adam`` on CPU (foreach off, no weight decay), float32, bit-exact:
    ``exp_avg.lerp_(g, 1-b1)`` = fma(w, g-m, m); ``exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)`` =
    fma((1-b2)*g, g, v*b2); ``denom = sqrt(v)/sqrt(1-b2^t) + eps``; ``p += (-lr/(1-b1^t) * m)/denom``."""
    p, g, m, v = (np.asarray(a, np.float32) for a in (p, g, m, v))
    m = _fmaf(np.float32(1 - beta1), g - m, m)
    v = _fmaf(np.float32(1 - beta2) * g, g, v * np.float32(beta2))
    bc1 = 1 - beta1 ** step
    bc2s = (1 - beta2 ** step) ** 0.5
    denom = (np.sqrt(v) / np.float32(bc2s) + np.float32(eps)).astype(np.float32)
    p = (p + (np.float32(-lr / bc1) * m) / denom).astype(np.float32)
    return p, m, v
