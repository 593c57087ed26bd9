"""Evaluation of a structure (a11): dSCC = Spearman of the triu true vs predicted distances.

Reference: HiC-GNN_main.py:135-139 (``spearmanr(dist_truth, cdist(coords)[triu])``) and
HiC_GAT_generalize_directly.py:242.  Ranks use scipy's tie rule (average rank of a tie group), so
the value equals scipy.stats.spearmanr on the same float32 distances; computed on the GPU.
"""
import torch

from . import ops


def _avg_rank(v):
    """Average ranks (1-based) with ties sharing their mean rank, in float64."""
    order = torch.argsort(v, stable=True)
    sv = v[order]
    n = v.numel()
    new_grp = torch.ones(n, dtype=torch.bool, device=v.device)
    new_grp[1:] = sv[1:] != sv[:-1]
    gid = torch.cumsum(new_grp.long(), 0) - 1
    pos = torch.arange(1, n + 1, dtype=torch.float64, device=v.device)
    ngrp = int(gid[-1].item()) + 1
    s = torch.zeros(ngrp, dtype=torch.float64, device=v.device).index_add_(0, gid, pos)
    c = torch.zeros(ngrp, dtype=torch.float64, device=v.device).index_add_(0, gid, torch.ones_like(pos))
    r = torch.empty(n, dtype=torch.float64, device=v.device)
    r[order] = (s / c)[gid]
    return r


def pearson(a, b):
    a = a.double() - a.double().mean()
    b = b.double() - b.double().mean()
    return float((a * b).sum() / torch.sqrt((a * a).sum() * (b * b).sum()))


def spearman(a, b):
    return pearson(_avg_rank(a), _avg_rank(b))


def triu_pairs(mat):
    n = mat.shape[0]
    idx = torch.triu_indices(n, n, offset=1, device=mat.device)
    return mat[idx[0], idx[1]]


def dscc(coords, truth):
    """HiC-GNN_main.py:135-139 on the GPU. ``truth`` is the [N, N] target (any float dtype)."""
    with torch.no_grad():
        d = ops.pairwise_dist(coords.detach())
        return spearman(triu_pairs(truth), triu_pairs(d))
