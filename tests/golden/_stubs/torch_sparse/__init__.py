"""Stub of ``torch_sparse`` 0.6.11: ``SparseTensor`` (COO -> sorted/coalesced CSR,
``to_symmetric`` (sum), ``sum(dim=0)``) and ``matmul`` (sparse x diag-sparse, sparse x dense sum)."""
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

    def sum(self, dim):
        """torch_sparse.reduce.sum: dim 0 -> scatter_add of the values by column (CSR order)."""
        if dim != 0:
            raise NotImplementedError
        v = self.storage.value()
        return torch.zeros(self.n, dtype=v.dtype).scatter_add_(0, self.storage.col(), v)

    def to_symmetric(self):
        r, c = self._row, self.storage.col()
        v = self.storage.value()
        vv = None if v is None else torch.cat([v, v])
        return SparseTensor(torch.cat([r, c]), torch.cat([c, r]), vv, (self.n, self.n))


def matmul(src, other, reduce="sum"):
    """torch_sparse.matmul for the two uses in layers.py: diag-sparse @ sparse (spspmm; each
    output entry is a single product) and sparse @ dense with reduce sum/add (spmm_sum: every row
    accumulated sequentially in CSR order, multiply then add)."""
    rp, c, v = src.storage.rowptr(), src.storage.col(), src.storage.value()
    if isinstance(other, SparseTensor):
        orp, oc, ov = other.storage.rowptr(), other.storage.col(), other.storage.value()
        rows, cols, vals = [], [], []
        for i in range(src.n):
            for e in range(int(rp[i]), int(rp[i + 1])):
                k = int(c[e])
                if k >= other.n:
                    continue
                for f in range(int(orp[k]), int(orp[k + 1])):
                    rows.append(i)
                    cols.append(int(oc[f]))
                    vals.append(v[e] * ov[f])
        val = torch.stack(vals) if vals else torch.zeros(0, dtype=ov.dtype)
        return SparseTensor(torch.tensor(rows), torch.tensor(cols), val, (other.n, other.n))
    if reduce not in ("sum", "add"):
        raise NotImplementedError(reduce)
    out = []
    for i in range(src.n):
        acc = torch.zeros(other.shape[1], dtype=other.dtype)
        for e in range(int(rp[i]), int(rp[i + 1])):
            acc = acc + v[e] * other[int(c[e])]
        out.append(acc)
    return torch.stack(out)
