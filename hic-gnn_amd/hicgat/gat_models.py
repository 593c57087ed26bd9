"""The in-scope HiC-GNN models on the HIP path, with the reference's forward()/get_model() surface.

* ``GATNetSelectiveResidualsUpdated``       -- models.py:614-691 (flagship, 601 475 parameters).
* ``GATNetHeadsChanged3LayersLeakyReLUv2``  -- models.py:1010-1047 (411 651 parameters).
* ``Net``                                   -- models.py:14-55, the SAGEConv baseline (697 475).

Submodules are registered in the reference's order (so the same seed gives the same initial
weights and the same state_dict keys).  ``forward`` returns the N x N distance matrix like the
reference (``cdist`` on the GPU); ``get_model`` returns the N x 3 coordinates; ``loss`` is the
fused path used by the training loop (distance + MSE [+ Pearson] without materialising N x N).
"""
import torch
import torch.nn.functional as F
from torch.nn import LayerNorm, Linear

from . import ops
from .nn import GATConv, SAGEConv


def _lin(layer, x):
    """A torch.nn.Linear of the model, run on the MFMA GEMM kernels."""
    return ops.linear(x, layer.weight, layer.bias)


class _CoordsModel(torch.nn.Module):
    def flat_parameters(self):
        """Parameter order for ``FlatAdam``'s flat buffers (default: ``parameters()``)."""
        return list(self.parameters())

    def forward(self, x, edge_index):
        return ops.pairwise_dist(self.get_model(x, edge_index))

    def loss(self, x, edge_index, truth, kind="mse", tile_range=(0, -1), stats=None):
        """Fused ``criterion(model(x, ei), truth)``; returns ``(loss, stats, coords)``."""
        coords = self.get_model(x, edge_index)
        loss, stats = ops.fused_dist_loss(coords, truth, kind, tile_range, stats)
        return loss, stats, coords


class GATNetSelectiveResidualsUpdated(_CoordsModel):
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

    conv_act = "relu"   # the relu of models.py:637 runs in the GAT aggregation's epilogue

    def flat_parameters(self):
        """dense* / align_dense* weights and biases adjacent in the flat buffers, so each residual
        block's [W1; W2] and [b1; b2] are views (one GEMM / one column sum in the backward)."""
        return [self.conv.lin_l.weight, self.conv.att_l, self.conv.att_r, self.conv.bias,
                self.densea.weight, self.align_densea.weight, self.densea.bias, self.align_densea.bias,
                self.norm_a.weight, self.norm_a.bias,
                self.dense1.weight, self.align_dense1.weight, self.dense1.bias, self.align_dense1.bias,
                self.norm1.weight, self.norm1.bias,
                self.dense2.weight, self.dense2.bias, self.norm2.weight, self.norm2.bias,
                self.dense3.weight, self.dense3.bias]

    def post_act(self, x):
        """models.py:638-659 (after the relu): each residual block relu(norm(dense(x))) +
        align_dense(x) as one fused op (one GEMM over [W; W_align], one row pass);
        relu(norm2(dense2(.))); dense3.  On graphs of >= ops.FUSED_TAIL_MIN_M rows the whole forward
        is one kernel (ops.fused_tail, tail_fused.hip) with the same backward."""
        if ops.fused_tail_ok(self, x):
            return ops.fused_tail(self, x)
        x = ops.dual_ln_relu_res(x, self.densea, self.align_densea, self.norm_a)
        x = ops.dual_ln_relu_res(x, self.dense1, self.align_dense1, self.norm1)
        x = ops.ln_relu_res(_lin(self.dense2, x), self.norm2)
        return _lin(self.dense3, x)

    def tail(self, x):
        """models.py:637-659 after the GATConv output."""
        return self.post_act(F.relu(x))

    def get_model(self, x, edge_index):
        return self.post_act(self.conv(x, edge_index, act=self.conv_act))


class GATNetHeadsChanged3LayersLeakyReLUv2(_CoordsModel):
    def __init__(self):
        super().__init__()
        self.conv = GATConv(512, 256, heads=2, concat=True)
        self.densea = Linear(512, 256)
        self.dense1 = Linear(256, 64)
        self.dense2 = Linear(64, 3)

    conv_act = None     # leaky_relu(0.01) stays a torch op on the GATConv output

    def tail(self, x):
        x = F.leaky_relu(x)
        x = F.leaky_relu(_lin(self.densea, x))
        x = F.leaky_relu(_lin(self.dense1, x))
        return _lin(self.dense2, x)

    post_act = tail

    def get_model(self, x, edge_index):
        return self.tail(self.conv(x, edge_index))


class Net(_CoordsModel):
    """models.py:14-55: SAGEConv(512, 512) -> relu -> 512-256-128-64-3 with relu between."""

    def __init__(self):
        super().__init__()
        self.conv = SAGEConv(512, 512)
        self.densea = Linear(512, 256)
        self.dense1 = Linear(256, 128)
        self.dense2 = Linear(128, 64)
        self.dense3 = Linear(64, 3)

    def get_model(self, x, edge_index):
        x = F.relu(self.conv(x, edge_index))
        x = F.relu(_lin(self.densea, x))
        x = F.relu(_lin(self.dense1, x))
        x = F.relu(_lin(self.dense2, x))
        return _lin(self.dense3, x)


MODELS = {
    "GATNetSelectiveResidualsUpdated": GATNetSelectiveResidualsUpdated,
    "GATNetHeadsChanged3LayersLeakyReLUv2": GATNetHeadsChanged3LayersLeakyReLUv2,
    "Net": Net,
}
