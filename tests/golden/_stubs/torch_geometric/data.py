"""Stub of ``torch_geometric.data.Data``: a plain attribute bag."""


class Data:
    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)
