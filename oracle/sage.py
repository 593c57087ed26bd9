"""Oracle: the reference's ``SAGEConv`` and the baseline model ``Net`` (TEST INFRASTRUCTURE ONLY).

SURVEY.md section 8 row f1.  ``layers.py:12-79`` builds on two third-party calls that are not
vendored or installed here (``torch_sparse==0.6.11``: ``SparseTensor.sum(dim=0)`` and
``matmul``), restated from their published CPU kernels:

  s_i    = sum over the CSR entries with column i of w     (adj_t.sum(dim=0): scatter_add in CSR
           order, float32 -- rows ascending for every column)                       layers.py:42
  inv_i  = 1 / s_i  (float32)                                                      layers.py:43-44
  n_ij   = inv_i * w_ij   (spspmm of diag(inv) and adj_t: one product per entry)   layers.py:49-52
  agg_i  = sum_e n_e * x[col_e]  (spmm_sum: sequential over row i, mul then add)   layers.py:74-77
  out    = lin_l(agg) + lin_r(x.long().float())   (lin_r has no bias)              layers.py:58-66

``SAGEConv.__init__`` never calls ``reset_parameters`` (``self.reset_parameters`` without the call,
``layers.py:33``), so the weights are torch.nn.Linear's own init in construction order: lin_l
(weight, bias), lin_r (weight).  ``Net`` (models.py:14-55): conv -> relu -> densea -> relu ->
dense1 -> relu -> dense2 -> relu -> dense3 (-> cdist in ``forward``).

``adj`` here is ``(rowptr, col, value)``: the int64 CSR and float32 networkx weights that
``utils.load_input`` produces (``oracle.graph.csr_from_matrix``), without self loops.
"""
import numpy as np
import torch
from torch.nn import Linear

from . import gat as _gat


def degree_inverse(rowptr, col, value, n):
    """layers.py:41-44: 1 / adj_t.sum(dim=0) in float32 (scatter in CSR order)."""
    s = np.zeros(n, dtype=np.float32)
    np.add.at(s, np.asarray(col), np.asarray(value, dtype=np.float32))
    with np.errstate(divide="ignore"):
        return np.float32(1.0) / s


def sage_aggregate(x, rowptr, col, value):
    """layers.py:46-52 + 74-77: matmul(diag(inv) @ adj_t, x, reduce='add') in float32.

    Entry k of every row is added in step k, so each row's sum runs sequentially in CSR order."""
    rowptr = torch.as_tensor(rowptr, dtype=torch.long)
    col = torch.as_tensor(col, dtype=torch.long)
    n = rowptr.numel() - 1
    inv = torch.tensor(degree_inverse(rowptr.numpy(), col.numpy(), value, n))
    deg = rowptr[1:] - rowptr[:-1]
    row = torch.repeat_interleave(torch.arange(n), deg)
    nv = inv[row] * torch.as_tensor(value, dtype=torch.float32)
    out = torch.zeros((n, x.shape[1]), dtype=x.dtype)
    maxdeg = int(deg.max()) if n else 0
    for k in range(maxdeg):
        rows = torch.nonzero(deg > k).flatten()
        e = rowptr[rows] + k
        out[rows] = out[rows] + nv[e].to(x.dtype)[:, None] * x[col[e]]
    return out


class _SageAggFn(torch.autograd.Function):
    """agg = N x with N = diag(inv) A (constant); d x = N^T d agg."""

    @staticmethod
    def forward(ctx, x, rowptr, col, value):
        ctx.save_for_backward(rowptr, col, value)
        return sage_aggregate(x, rowptr, col, value)

    @staticmethod
    def backward(ctx, g):
        rowptr, col, value = ctx.saved_tensors
        n = rowptr.numel() - 1
        inv = torch.tensor(degree_inverse(rowptr.numpy(), col.numpy(), value.numpy(), n))
        row = torch.repeat_interleave(torch.arange(n), rowptr[1:] - rowptr[:-1])
        nv = inv[row] * value.float()
        dx = torch.zeros_like(g).index_add_(0, col, nv[:, None] * g[row])
        return dx, None, None, None


class SAGEConv(torch.nn.Module):
    def __init__(self, in_channels, out_channels, normalize=False, root_weight=True, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.normalize, self.root_weight = normalize, root_weight
        self.lin_l = Linear(in_channels, out_channels, bias=bias)
        if root_weight:
            self.lin_r = Linear(in_channels, out_channels, bias=False)

    def forward(self, x, adj):
        rowptr, col, value = (torch.as_tensor(a) for a in adj)
        out = self.lin_l(_SageAggFn.apply(x, rowptr, col, value.float()).float())
        if self.root_weight:
            out = out + self.lin_r(x.long().float())
        if self.normalize:
            out = torch.nn.functional.normalize(out, p=2.0, dim=-1)
        return out


class Net(torch.nn.Module):
    """models.py:14-55."""

    def __init__(self):
        super().__init__()
        self.conv = SAGEConv(512, 512)
        self.densea = Linear(512, 256)
        self.dense1 = Linear(256, 128)
        self.dense2 = Linear(128, 64)
        self.dense3 = Linear(64, 3)

    def get_model(self, x, adj):
        x = self.conv(x, adj).relu()
        x = self.densea(x).relu()
        x = self.dense1(x).relu()
        x = self.dense2(x).relu()
        return self.dense3(x)

    def forward(self, x, adj):
        c = self.get_model(x, adj)
        return torch.cdist(c, c, p=2, compute_mode=_gat.CDIST_MODE)
