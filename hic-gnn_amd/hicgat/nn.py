"""``GATConv``: drop-in for PyG 1.7.2 ``torch_geometric.nn.GATConv`` on the HIP kernels.

Same constructor arguments, parameter names and state_dict keys as the version the reference
instantiates (``models.py:619``: ``GATConv(512, 256, heads=2, concat=True)``):
``lin_l.weight`` [H*C, F] (no bias; ``lin_r`` is the same module, so ``lin_r.weight`` aliases it
in the state_dict exactly like PyG), ``att_l`` / ``att_r`` [1, H, C], ``bias`` [H*C].  The RNG
draws of the initialisation follow PyG 1.7.2 (``torch.nn.Linear``'s own init, then glorot on
lin_l, glorot on lin_r (the same tensor), glorot on att_l, att_r, zeros on bias), so
``torch.manual_seed(s)`` gives the reference's initial weights bit for bit.
"""
import math

import torch
from torch.nn import Linear, Parameter

from . import ops


def _glorot(t):
    stdv = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-stdv, stdv)


class GATConv(torch.nn.Module):
    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2,
                 dropout=0.0, add_self_loops=True, bias=True, **kwargs):
        super().__init__()
        if not isinstance(in_channels, int):
            raise NotImplementedError("bipartite (tuple) in_channels is out of scope")
        if not concat:
            raise NotImplementedError("concat=False (head mean) is out of scope")
        if dropout != 0.0:
            raise NotImplementedError("attention dropout > 0 is out of scope (the reference uses 0)")
        if not add_self_loops:
            raise NotImplementedError("add_self_loops=False is out of scope")
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope = concat, negative_slope
        self.dropout, self.add_self_loops = dropout, add_self_loops
        self.lin_l = Linear(in_channels, heads * out_channels, bias=False)
        self.lin_r = self.lin_l
        self.att_l = Parameter(torch.Tensor(1, heads, out_channels))
        self.att_r = Parameter(torch.Tensor(1, heads, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(heads * out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        _glorot(self.lin_l.weight)
        _glorot(self.lin_r.weight)
        _glorot(self.att_l)
        _glorot(self.att_r)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x, edge_index, act=None):
        """``edge_index`` is a ``hicgat.graph.Adj`` (the reference passes a SparseTensor).
        ``act="relu"`` (not in PyG) returns relu(forward(x)) with the relu fused into the kernel."""
        return ops.gat_conv(x, self.lin_l.weight, self.att_l, self.att_r, self.bias, edge_index,
                            self.negative_slope, act)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, heads={self.heads})"


class SAGEConv(torch.nn.Module):
    """Drop-in for the reference's own ``layers.SAGEConv`` (layers.py:12-79).

    Same parameters and state_dict keys (``lin_l.weight``, ``lin_l.bias``, ``lin_r.weight``) and
    the same init (torch.nn.Linear's, in construction order: the reference never calls its
    ``reset_parameters``, layers.py:33).  ``forward`` keeps the degree normalisation
    ``diag(1/colsum) @ adj`` and the ``x.long()`` truncation of the root branch (layers.py:64)."""

    def __init__(self, in_channels, out_channels, normalize=False, root_weight=True, bias=True, **kwargs):
        super().__init__()
        if not isinstance(in_channels, int):
            raise NotImplementedError("bipartite (tuple) in_channels is out of scope")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.normalize, self.root_weight = normalize, root_weight
        self.lin_l = Linear(in_channels, out_channels, bias=bias)
        if root_weight:
            self.lin_r = Linear(in_channels, out_channels, bias=False)

    def reset_parameters(self):
        self.lin_l.reset_parameters()
        if self.root_weight:
            self.lin_r.reset_parameters()

    def forward(self, x, edge_index):
        out = ops.sage_conv(x, self.lin_l.weight, self.lin_l.bias,
                            self.lin_r.weight if self.root_weight else None, edge_index)
        if self.normalize:
            out = torch.nn.functional.normalize(out, p=2.0, dim=-1)
        return out

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"
