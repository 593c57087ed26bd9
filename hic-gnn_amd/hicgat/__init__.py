"""hicgat -- the GAT-HiC per-epoch hot path on MI355X (gfx950) HIP kernels.

Drop-in surface of the reference (beyzoskaya/HiC-GNN):
  hicgat.nn.GATConv                           ~ torch_geometric.nn.GATConv (PyG 1.7.2)
  hicgat.nn.SAGEConv                          ~ layers.SAGEConv (layers.py:12-79)
  hicgat.gat_models.GATNetSelectiveResidualsUpdated / GATNetHeadsChanged3LayersLeakyReLUv2 / Net
                                              ~ models.py:614-691 / :1010-1047 / :14-55
  hicgat.graph.load_input / cont2dist / convert_to_matrix / Adj
                                              ~ utils.py:10-80 (+ torch_sparse.SparseTensor)
  hicgat.train.train / main                   ~ HiC-GNN_main.py:107-160
  hicgat.metrics.dscc, hicgat.io.write_pdb    ~ HiC-GNN_main.py:135-139, utils.WritePDB
  hicgat.kr.KRnorm                            ~ r_utils.R:1-93 (normalize.R)
  hicgat.align.domain_alignment / generalize  ~ utils.py:83-109, HiC_GAT_generalize_directly.py:312-336
  hicgat.embed.node2vec                       ~ Node2Vec(...).fit(...) at HiC_GAT_generalize_directly.py:150-155
Compute runs in libhicgat.so (include/hicgat.h); there is no CPU fallback.
"""
from . import _lib, align, dist, embed, graph, graphs, io, kernels, kr, metrics, nn, ops, optim, synth, train  # noqa: F401
from .gat_models import (GATNetHeadsChanged3LayersLeakyReLUv2,  # noqa: F401
                         GATNetSelectiveResidualsUpdated, MODELS, Net)
from .graph import Adj, Data, Truth, cont2dist, convert_to_matrix, load_input  # noqa: F401
from .nn import GATConv, SAGEConv  # noqa: F401
from .optim import FlatAdam  # noqa: F401

__version__ = "0.1.0"
