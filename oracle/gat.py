"""Oracle: PyG 1.7.2 ``GATConv`` and the two in-scope GAT-HiC models (TEST INFRASTRUCTURE ONLY).

``GATConv`` is third-party (``torch_geometric==1.7.2``, ``requirements.txt:37``), not vendored in
the reference and not installed here, so its algorithm is restated from the published 1.7.2 code
path that ``models.py:619`` (``GATConv(512, 256, heads=2, concat=True)``) takes with a SparseTensor
``edge_index``:

  h = lin_l(x) (no bias; lin_r *is* lin_l), a_l = <h, att_l>, a_r = <h, att_r> per head;
  adj = set_diag(adj);  e_ij = leaky_relu(a_l[j] + a_r[i], 0.2) for CSR row i (dst), col j (src);
  alpha = exp(e - segment_max_i) / (segment_sum_i + 1e-16)   (torch_geometric.utils.softmax, ptr path)
  out_i = segment_csr_sum_j(h_j * alpha_ij);  out = out.view(N, H*C) + bias.

Parameter construction order (and hence RNG consumption) follows 1.7.2: ``torch.nn.Linear`` (its
own kaiming init), then ``reset_parameters``: glorot(lin_l.weight), glorot(lin_r.weight) (the same
tensor, drawn twice), glorot(att_l), glorot(att_r), zeros(bias).
"""
import math

import torch
import torch.nn.functional as F
from torch.nn import LayerNorm, Linear


# torch.cdist compute mode of the models' forward.  The reference uses the default, which takes the
# matrix-multiply formula for N > 25 (non-zero diagonal, O(1e-4) absolute error
# on small distances, noise in the gradients).  Tests that compare against the exact-distance HIP
# kernels switch it to "donot_use_mm_for_euclid_dist".
CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"


def glorot(t):
    stdv = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-stdv, stdv)


def set_diag(rowptr, col):
    """torch_sparse 0.6.11 ``set_diag`` (values=None) on an int64 CSR, O(nnz) like its C++ kernel.

    Existing diagonal entries are dropped (``remove_diag``) and one (i, i) entry is inserted into
    every row at its sorted position (``non_diag_mask``).  Returns the new ``(rowptr, col)``.
    """
    n = rowptr.numel() - 1
    row = torch.repeat_interleave(torch.arange(n), rowptr[1:] - rowptr[:-1])
    keep = row != col
    row, col = row[keep], col[keep]
    deg = torch.zeros(n, dtype=torch.long).index_add(0, row, torch.ones_like(row))
    below = torch.zeros(n, dtype=torch.long).index_add(0, row, (col < row).long())
    new_ptr = torch.zeros(n + 1, dtype=torch.long)
    new_ptr[1:] = torch.cumsum(deg + 1, 0)
    old_ptr = torch.zeros(n + 1, dtype=torch.long)
    old_ptr[1:] = torch.cumsum(deg, 0)
    pos = torch.arange(row.numel()) - old_ptr[row] + new_ptr[row] + (col > row).long()
    out = torch.empty(row.numel() + n, dtype=torch.long)
    out[pos] = col
    out[new_ptr[:-1] + below] = torch.arange(n)
    return new_ptr, out


def gat_softmax_aggregate(h, a_l, a_r, rowptr, col, negative_slope=0.2):
    """PyG 1.7.2 message/softmax/aggregate over a CSR that already holds the self loops.

    ``h`` [N, H, C], ``a_l``/``a_r`` [N, H], ``rowptr``/``col`` int64 tensors.  Returns [N, H, C].
    The [nnz, H, C] message tensor is materialised exactly like the reference path.
    """
    n = h.shape[0]
    deg = rowptr[1:] - rowptr[:-1]
    row = torch.repeat_interleave(torch.arange(n), deg)
    e = F.leaky_relu(a_l[col] + a_r[row], negative_slope)                   # [nnz, H]
    idx = row.view(-1, 1).expand_as(e)
    e_max = torch.full((n, e.shape[1]), float("-inf"), dtype=e.dtype).scatter_reduce(
        0, idx, e, reduce="amax", include_self=True)
    u = (e - e_max[row]).exp()
    u_sum = torch.zeros((n, e.shape[1]), dtype=e.dtype).index_add(0, row, u)
    alpha = u / (u_sum[row] + 1e-16)
    msg = h[col] * alpha.unsqueeze(-1)                                      # [nnz, H, C]
    return torch.zeros_like(h).index_add(0, row, msg)


class GATConv(torch.nn.Module):
    """PyG 1.7.2 ``GATConv`` restated (SparseTensor input, dropout 0, self loops on)."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True):
        super().__init__()
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope = concat, negative_slope
        self.dropout, self.add_self_loops = dropout, add_self_loops
        self.lin_l = Linear(in_channels, heads * out_channels, bias=False)
        self.lin_r = self.lin_l
        self.att_l = torch.nn.Parameter(torch.Tensor(1, heads, out_channels))
        self.att_r = torch.nn.Parameter(torch.Tensor(1, heads, out_channels))
        if bias and concat:
            self.bias = torch.nn.Parameter(torch.Tensor(heads * out_channels))
        elif bias:
            self.bias = torch.nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.lin_l.weight)
        glorot(self.lin_r.weight)
        glorot(self.att_l)
        glorot(self.att_r)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x, adj):
        """``adj`` = (rowptr, col) int64 tensors of the symmetric CSR (``utils.py:70-71``)."""
        rowptr, col = adj
        if self.add_self_loops:
            rowptr, col = set_diag(rowptr, col)
        H, C = self.heads, self.out_channels
        h = self.lin_l(x).view(-1, H, C)
        a_l = (h * self.att_l).sum(dim=-1)
        a_r = (h * self.att_r).sum(dim=-1)
        out = gat_softmax_aggregate(h, a_l, a_r, rowptr, col, self.negative_slope)
        out = out.reshape(-1, H * C) if self.concat else out.mean(dim=1)
        if self.bias is not None:
            out = out + self.bias
        return out


class GATNetSelectiveResidualsUpdated(torch.nn.Module):
    """Restates ``models.py:614-691`` (flagship; 601 475 parameters)."""

    def __init__(self):
        super().__init__()
        self.conv = GATConv(512, 256, heads=2, concat=True)
        self.densea = Linear(512, 256)
        self.norm_a = LayerNorm(256)
        self.align_densea = Linear(512, 256)
        self.dense1 = Linear(256, 128)
        self.norm1 = LayerNorm(128)
        self.align_dense1 = Linear(256, 128)
        self.dense2 = Linear(128, 64)
        self.norm2 = LayerNorm(64)
        self.dense3 = Linear(64, 3)

    def get_model(self, x, adj):
        x = F.relu(self.conv(x, adj))
        r = self.align_densea(x)
        x = F.relu(self.norm_a(self.densea(x))) + r
        r = self.align_dense1(x)
        x = F.relu(self.norm1(self.dense1(x))) + r
        x = F.relu(self.norm2(self.dense2(x)))
        return self.dense3(x)

    def forward(self, x, adj):
        c = self.get_model(x, adj)
        return torch.cdist(c, c, p=2, compute_mode=CDIST_MODE)


class GATNetHeadsChanged3LayersLeakyReLUv2(torch.nn.Module):
    """Restates ``models.py:1010-1047`` (411 651 parameters)."""

    def __init__(self):
        super().__init__()
        self.conv = GATConv(512, 256, heads=2, concat=True)
        self.densea = Linear(512, 256)
        self.dense1 = Linear(256, 64)
        self.dense2 = Linear(64, 3)

    def get_model(self, x, adj):
        x = F.leaky_relu(self.conv(x, adj))
        x = F.leaky_relu(self.densea(x))
        x = F.leaky_relu(self.dense1(x))
        return self.dense2(x)

    def forward(self, x, adj):
        c = self.get_model(x, adj)
        return torch.cdist(c, c, p=2, compute_mode=CDIST_MODE)


MODELS = {
    "GATNetSelectiveResidualsUpdated": GATNetSelectiveResidualsUpdated,
    "GATNetHeadsChanged3LayersLeakyReLUv2": GATNetHeadsChanged3LayersLeakyReLUv2,
}
