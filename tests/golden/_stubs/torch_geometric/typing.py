"""Stub of ``torch_geometric.typing`` (type aliases only)."""
from typing import Optional, Tuple, Union

from torch import Tensor

OptTensor = Optional[Tensor]
OptPairTensor = Tuple[Tensor, OptTensor]
Adj = Union[Tensor, object]
Size = Optional[Tuple[int, int]]
