"""Stub of ``torch_sparse.SparseTensor``: COO -> sorted/coalesced CSR, ``to_symmetric`` (sum)."""
import numpy as np
import torch


class _Storage:
    def __init__(self, rowptr, col, value):
        self._rowptr, self._col, self._value = rowptr, col, value

    def rowptr(self):
        return self._rowptr

    def col(self):
        return self._col

    def value(self):
        return self._value


class SparseTensor:
    def __init__(self, row, col, value=None, sparse_sizes=None):
        row = torch.as_tensor(row, dtype=torch.long)
        col = torch.as_tensor(col, dtype=torch.long)
        self.init_row, self.init_col = row.clone(), col.clone()
        n = int(sparse_sizes[0]) if sparse_sizes is not None else int(row.max()) + 1
        self.n = n
        key = (row * n + col).numpy()
        order = np.argsort(key, kind="stable")
        key = key[order]
        uniq, start = np.unique(key, return_index=True)
        if value is not None:
            v = torch.as_tensor(value)[torch.as_tensor(order)]
            vsum = torch.zeros(len(uniq), dtype=v.dtype).index_add(
                0, torch.as_tensor(np.repeat(np.arange(len(uniq)), np.diff(np.append(start, len(key))))), v)
        else:
            vsum = None
        r = torch.as_tensor(uniq // n)
        c = torch.as_tensor(uniq % n)
        rowptr = torch.zeros(n + 1, dtype=torch.long)
        rowptr[1:] = torch.cumsum(torch.bincount(r, minlength=n), 0)
        self.storage = _Storage(rowptr, c, vsum)
        self._row = r

    def to_symmetric(self):
        r, c = self._row, self.storage.col()
        v = self.storage.value()
        vv = None if v is None else torch.cat([v, v])
        return SparseTensor(torch.cat([r, c]), torch.cat([c, r]), vv, (self.n, self.n))


def matmul(*a, **k):
    raise NotImplementedError("torch_sparse.matmul is out of scope for the GAT fixtures")
