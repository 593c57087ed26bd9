"""Stub of ``torch_geometric.nn``: GATConv = the oracle's PyG 1.7.2 restatement."""
import torch

from oracle.gat import GATConv as _OracleGATConv


class GATConv(_OracleGATConv):
    def forward(self, x, edge_index):
        st = edge_index.storage
        return super().forward(x, (st.rowptr(), st.col()))


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", **kwargs):
        super().__init__()
        self.aggr = aggr

    def propagate(self, edge_index, size=None, **kwargs):
        """PyG 1.7.2 fused path for a SparseTensor adjacency: message_and_aggregate(adj_t, ...)."""
        return self.message_and_aggregate(edge_index, **kwargs)


class GCNConv(torch.nn.Module):
    def __init__(self, *a, **k):
        raise NotImplementedError("GCNConv is out of scope")
