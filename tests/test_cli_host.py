"""CPU: the host logic of the training / generalisation drivers and of the truth target.

* ``hicgat.train.main`` follows HiC-GNN_main.py: default conversions ``[.1,.1,2]`` (:33), every
  conversion trains a fresh model against ``cont2dist(y, 0.5)`` (:120), the best dSCC wins
  (list.index(max)), the log lines of :155-156, node2vec fed the ZERO-DIAGONAL matrix (the saved
  ``*_matrix.txt`` of HiC_GAT_generalize_directly.py:113-115,150-155).  The device steps are
  replaced by recording stand-ins (this checks the driver, not the kernels).
* the saved weights are plain CPU tensors that load into the oracle model with a bare torch.load;
* an asymmetric target folded into ``graph.Truth``'s symmetric form keeps the MSE and its gradient.
"""
import os

import numpy as np
import pytest
import torch


def _tiny_list(tmp_path):
    rng = np.random.default_rng(3)
    rows = []
    for i in range(12):
        for j in range(i, 12):
            if rng.random() < 0.6 or j == i + 1:
                rows.append((i * 1000, j * 1000, float(rng.integers(1, 30))))
    p = tmp_path / "tiny_list.txt"
    np.savetxt(p, np.array(rows))
    return str(p)


class _FakeModel(torch.nn.Module):
    made = 0

    def __init__(self):
        super().__init__()
        _FakeModel.made += 1
        self.k = _FakeModel.made
        self.w = torch.nn.Parameter(torch.randn(3))

    def to(self, *a, **k):
        return self

    def get_model(self, x, ei):
        return torch.zeros(x.shape[0], 3) + self.k


def test_train_main_follows_reference_driver(tmp_path, monkeypatch):
    from hicgat import embed, graph, metrics
    from hicgat import train as T
    seen = {"factors": [], "truth_ids": set(), "n2v_diag": None}

    class _Data:
        def __init__(self, x, y):
            self.x, self.y, self.edge_index = x, y, None

    def fake_load_input(mat, feats, device="cuda"):
        return _Data(torch.as_tensor(feats), torch.as_tensor(mat))

    def fake_from_contacts(y, factor):
        seen["factors"].append(factor)
        t = graph.Truth(torch.rand(y.shape[0], y.shape[0]).double().add(torch.eye(y.shape[0])))
        return t

    def fake_train(model, data, truth, lr, thresh, steps, loss):
        seen["truth_ids"].add(id(truth))
        return None, [1.0, 0.5, 0.25 / model.k]

    scores = {}

    def fake_dscc(coords, truth):
        k = int(coords[0, 0])
        scores[k] = [0.3, 0.9, 0.9, 0.2][(k - 1) % 4]
        return scores[k]

    def fake_node2vec(mat, seed=42, **kw):
        seen["n2v_diag"] = np.diag(np.asarray(mat)).copy()
        return torch.zeros(np.asarray(mat).shape[0], 8)

    monkeypatch.setattr(T.graph, "load_input", fake_load_input)
    monkeypatch.setattr(T.graph.Truth, "from_contacts", staticmethod(fake_from_contacts))
    monkeypatch.setattr(T, "train", fake_train)
    monkeypatch.setattr(T.metrics, "dscc", fake_dscc)
    monkeypatch.setattr(embed, "node2vec", fake_node2vec)
    monkeypatch.setitem(T.MODELS, "GATNetSelectiveResidualsUpdated", _FakeModel)
    _FakeModel.made = 0
    out = str(tmp_path / "run")
    assert T.main([_tiny_list(tmp_path), "node2vec", "--no-kr", "--out", out]) == 0
    conv = list(np.arange(0.1, 2, 0.1))                     # HiC-GNN_main.py:33 default, :51-52
    assert _FakeModel.made == len(conv) == 19
    assert seen["factors"] == [0.5]                         # one truth, cont2dist(y, 0.5) (:120)
    assert len(seen["truth_ids"]) == 1
    assert seen["n2v_diag"] is not None and not seen["n2v_diag"].any()
    with open(out + "_log.txt") as fh:
        lines = fh.read().splitlines()
    # first maximum (0.9 at the 2nd model), as tempspear.index(max(tempspear))
    assert lines[0] == f"Optimal conversion factor: {conv[1]}"
    assert lines[1] == "Optimal dSCC: 0.9"
    assert lines[2] == f"Final MSE loss: {0.25 / 2}"
    assert os.path.exists(out + "_structure.pdb")
    sd = torch.load(out + "_weights.pt")                    # bare load, as evaluate.py:87
    assert all(v.device.type == "cpu" for v in sd.values())
    assert metrics  # noqa


def test_parse_conversions():
    from hicgat.train import parse_conversions
    assert parse_conversions("[.5]") == [0.5]
    assert len(parse_conversions("[.1,.1,2]")) == 19
    with pytest.raises(ValueError):
        parse_conversions("[1, 2]")


def test_cpu_state_dict_roundtrip_into_oracle(tmp_path):
    """Weights saved from a FlatAdam-backed model (every parameter a view of one flat buffer) are
    independent CPU tensors and load into the oracle model under the PyG 1.7.2 key names."""
    import hicgat
    from hicgat.train import cpu_state_dict
    from oracle import gat as og
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated()
    hicgat.FlatAdam(model.flat_parameters())
    sd = cpu_state_dict(model)
    for v in sd.values():
        assert v.untyped_storage().nbytes() == v.numel() * v.element_size()
    p = tmp_path / "w.pt"
    torch.save(sd, p)
    ref = og.GATNetSelectiveResidualsUpdated()
    ref.load_state_dict(torch.load(p, weights_only=True))
    for (k, v), (k2, v2) in zip(sorted(model.state_dict().items()), sorted(ref.state_dict().items())):
        assert k == k2 and torch.equal(v, v2)


def test_asymmetric_truth_folded_keeps_mse_and_gradient():
    """graph.Truth's symmetric form of an asymmetric target: the full-matrix MSE of a distance
    matrix (zero diagonal) and its gradient are unchanged."""
    from hicgat import graph
    rng = np.random.default_rng(7)
    n = 37
    t = rng.random((n, n))
    t = (t + t.T) / 2
    np.fill_diagonal(t, 0)
    t[3, 9] += 1e-3                                   # asymmetric pairs, like R's rounding (and larger)
    t[20, 4] -= 2e-2
    t = t.astype(np.float32)
    tr = graph.Truth(torch.tensor(t))
    assert tr.asymmetric_source and tr.symmetric
    ts = tr.dense().double()
    assert torch.equal(ts, ts.t())
    c = torch.tensor(rng.random((n, 3)), dtype=torch.float64, requires_grad=True)

    def mse(T):
        d = torch.cdist(c, c)
        return ((d - T) ** 2).mean()
    l0 = mse(torch.tensor(t, dtype=torch.float64))
    g0, = torch.autograd.grad(l0, c)
    l1 = mse(ts)
    g1, = torch.autograd.grad(l1, c)
    assert abs(l1.item() - l0.item()) <= 1e-6 * l0.item()
    assert (g1 - g0).abs().max().item() <= 1e-6 * g0.abs().max().item()
