"""CPU, world_size 2 and 3 (gloo): the destination-row sharded step (hicgat.dist.ShardedTrainer),
in both forms ("slab": x replicated, no h / dout all-gathers; "allgather": the north star's h
all-gather), equals the single-rank step, and the single-rank step equals the autograd oracle.

The trainer runs against tests/cpu_kernels.CpuKernels (torch stand-ins for the HIP kernels), so
this covers the partition, the all-gathers / all-reduces and the manual backward bookkeeping; the
HIP kernels themselves are covered by tests/test_gpu_parity.py.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
STEPS = 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(n=300, seed=0, skew=False):
    """Random symmetric contacts; ``skew``: a dense band over the first fifth of the rows plus a
    sparse tail (equal-ROW shards would give rank 0 most of the edges)."""
    rng = np.random.default_rng(seed)
    p = np.full((n, n), 0.08)
    if skew:
        p[:] = 0.02
        p[:n // 5, :n // 5] = 0.9
    a = (rng.random((n, n)) < p) * rng.integers(1, 50, (n, n)).astype(np.float64)
    a = np.triu(a, 1)
    a = a + a.T
    a[17, :] = 0
    a[:, 17] = 0
    x = (0.1 * rng.standard_normal((n, 512))).astype(np.float32)
    return a, x


def _setup(n, skew=False):
    for p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd"), HERE):
        if p not in sys.path:
            sys.path.insert(0, p)
    import hicgat
    from oracle import graph as ogr
    a, x = _problem(n, skew=skew)
    iu = np.argwhere(np.triu(a != 0, 1))
    adj = hicgat.Adj(torch.tensor(iu[:, 0]), torch.tensor(iu[:, 1]), None, (n, n)).to_symmetric().to("cpu")
    truth = hicgat.Truth(ogr.cont2dist(torch.tensor(a), 0.5))
    return hicgat, adj, truth, torch.tensor(x)


def _worker(rank, world, port, n, kind, out, skew=False, mode="slab"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hicgat, adj, truth, x = _setup(n, skew)
        from cpu_kernels import CpuKernels, torch_tail
        torch_tail(hicgat)
        torch.manual_seed(0)
        model = hicgat.GATNetSelectiveResidualsUpdated()
        tr = hicgat.dist.ShardedTrainer(model, x, adj, truth, lr=1e-3, kind=kind, kern=CpuKernels(), mode=mode)
        # what this rank holds: its edges, its x rows, its support rows / entries, its slab entries
        sf = tr.sf
        held = torch.tensor([tr.local_nnz, tr.local_rows, tr.s1 - tr.s0,
                             int(sf.rowptr[tr.s1]) - int(sf.rowptr[tr.s0]), (tr.slab_nnz if tr.slab_nnz is not None else -1),
                             tr.t1 - tr.t0], dtype=torch.long)
        allheld = [torch.zeros_like(held) for _ in range(world)]
        dist.all_gather(allheld, held)
        losses, grad1, stats1 = [], None, None
        for _ in range(STEPS):
            loss, stats, _ = tr.step()
            losses.append(float(loss))
            if grad1 is None:
                grad1, stats1 = tr.opt.grad.clone(), stats.clone()   # all-reduced step-1 gradient
        if rank == 0:
            # per-parameter step-1 gradients by name (the flat layout follows model.flat_parameters())
            off, by_name = {}, {}
            for p, o in zip(tr.opt.params, tr.opt.offsets):
                off[id(p)] = o
            for name, p in model.named_parameters():
                by_name[name] = grad1[off[id(p)]:off[id(p)] + p.numel()].view_as(p).clone()
            torch.save({"losses": losses, "flat": tr.opt.flat.clone(), "grad1": grad1, "stats": stats1,
                        "grads": by_name, "held": torch.stack(allheld), "nnz": adj.device_nnz if hasattr(adj, "col32")
                        and adj.col32 is not None else -1, "truth_numel": truth.dense().numel()}, out)
    finally:
        dist.destroy_process_group()


def _run(world, n, kind, tmp_path, skew=False, mode="slab"):
    out = str(tmp_path / f"w{world}_{kind}_{int(skew)}{mode}.pt")
    mp.spawn(_worker, args=(world, _free_port(), n, kind, out, skew, mode), nprocs=world, join=True)
    return torch.load(out, weights_only=True)


def _close(a, b, stats_rtol=1e-9, loss_rtol=1e-6, grad_rtol=1e-5):
    """Step 1 (loss, moments, all-reduced gradient) agrees to summation-order rounding; later
    steps only loosely, because Adam normalises near-zero gradient entries (e.g. dense3.bias,
    whose exact gradient is 0 by translation invariance) into lr-sized moves of either sign.
    Shards of the same form share the forward bit for bit up to the coordinates (stats to 1e-9);
    the aggregate-first form rounds the GATConv output differently (fp32: the north star's 1e-5)."""
    assert abs(b["losses"][0] - a["losses"][0]) <= loss_rtol * abs(a["losses"][0])
    assert torch.allclose(b["stats"][:9], a["stats"][:9], rtol=stats_rtol, equal_nan=True)
    g1, g2 = a["grad1"], b["grad1"]
    assert (g2 - g1).abs().max().item() <= grad_rtol * g1.abs().max().item()
    np.testing.assert_allclose(b["losses"], a["losses"], rtol=1e-3)


@pytest.mark.parametrize("kind", ["mse", "combined", "contrastive"])
def test_sharded_step_equals_single_rank(tmp_path, kind):
    one = _run(1, 300, kind, tmp_path)
    two = _run(2, 300, kind, tmp_path)
    _close(one, two)


def test_aggregate_first_form_equals_h_first_form(tmp_path):
    """The "xagg" form (out = W (sum alpha x) + b, gat_xagg.hip) is the same layer as the h-first
    form regrouped: world 1 and world 2 xagg against world 1 slab."""
    one = _run(1, 300, "combined", tmp_path, mode="slab")
    tol = dict(stats_rtol=1e-5, loss_rtol=1e-5, grad_rtol=1e-4)
    _close(one, _run(1, 300, "combined", tmp_path, mode="xagg"), **tol)
    _close(one, _run(2, 300, "combined", tmp_path, mode="xagg"), **tol)


@pytest.mark.parametrize("mode", ["slab", "xagg", "allgather"])
def test_three_uneven_ranks_equal_single_rank(tmp_path, mode):
    """World 3 on a 301-node graph (uneven rows, edges, tiles and support rows per rank): both
    step forms equal the world-1 step; the shards partition the edges, the support and the tiles."""
    one = _run(1, 301, "combined", tmp_path, mode=mode)
    three = _run(3, 301, "combined", tmp_path, mode=mode)
    _close(one, three)
    held, full = three["held"], one["held"][0]
    assert int(held[:, 0].sum()) == int(full[0]) and int(held[:, 1].sum()) == 301
    assert int(held[:, 2].sum()) == 301 and int(held[:, 3].sum()) == int(full[3])
    assert int(held[:, 5].sum()) == int(full[5])
    if mode == "slab":
        assert int(held[:, 4].sum()) == int(full[4]) == int(full[0])     # the slabs partition the CSR


@pytest.mark.parametrize("world", [4, 8])
def test_auto_form_at_four_and_eight_ranks_equals_single_rank(tmp_path, world):
    """bench.py's default form at the driver's larger world sizes ("auto" = xagg from 2 ranks,
    hicgat.dist.resolve_mode): 4 and 8 gloo ranks on a 301-node graph equal world 1 of the same
    form, and the shards still partition the rows, edges, tiles and support rows."""
    from hicgat import dist as hdist
    assert hdist.resolve_mode("auto", world) == "xagg" and hdist.resolve_mode("auto", 2) == "xagg"
    assert hdist.resolve_mode("auto", 1) == "slab"
    one = _run(1, 301, "combined", tmp_path, mode="xagg")
    many = _run(world, 301, "combined", tmp_path, mode="auto")
    _close(one, many)
    held, full = many["held"], one["held"][0]
    assert held.shape[0] == world
    assert int(held[:, 0].sum()) == int(full[0]) and int(held[:, 1].sum()) == 301
    assert int(held[:, 2].sum()) == 301 and int(held[:, 3].sum()) == int(full[3])
    assert int(held[:, 5].sum()) == int(full[5])     # (the xagg form has no slab structure: column 4 is -1)


@pytest.mark.parametrize("kind", ["mse", "contrastive"])
def test_single_rank_sharded_step_equals_autograd_oracle(tmp_path, kind):
    """The manual backward of ShardedTrainer (CpuKernels, P = 1) vs the oracle model trained by
    autograd + torch Adam with exact distances: same losses, same parameters.  "contrastive": the
    f5 loss (train_and_test_same_res_GAT_node2vec.py:107-134) through the background + support form."""
    one = _run(1, 300, kind, tmp_path)
    hicgat, adj, truth, x = _setup(300)
    from oracle import gat as og
    from oracle import loop as ol
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        torch.manual_seed(0)
        ref = og.GATNetSelectiveResidualsUpdated()
        radj = (adj.storage.rowptr(), adj.storage.col())
        hist = ol.train(ref, x, radj, truth.dense().double(), steps=STEPS, loss=kind)
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    assert abs(one["losses"][0] - hist[0]) <= 1e-6 * hist[0]
    np.testing.assert_allclose(one["losses"], hist, rtol=1e-3)
    # step-1 gradients of the manual backward vs autograd (the oracle's params after 1 step would
    # mix in Adam's sign sensitivity; recompute the oracle's first gradient instead)
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        torch.manual_seed(0)
        ref = og.GATNetSelectiveResidualsUpdated()
        if kind == "contrastive":
            ol.contrastive_loss(ref.get_model(x, radj), truth.dense().double()).backward()
        else:
            ol.mse_loss(ref(x, radj), truth.dense().double()).backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    model = hicgat.GATNetSelectiveResidualsUpdated()
    for (name, p), pr in zip(model.named_parameters(), ref.parameters()):
        mine = one["grads"][name]
        scale = pr.grad.abs().max().item()
        if name == "dense3.bias":   # exact value 0 (translation invariance): rounding noise only
            assert mine.abs().max().item() < 1e-6 * max(1.0, scale)
            continue
        assert (mine - pr.grad).abs().max().item() <= 1e-4 * scale, name


@pytest.mark.parametrize("mode", ["slab", "xagg", "allgather"])
def test_skewed_graph_shards_balance_nnz_and_match_world1(tmp_path, mode):
    """destination rows split by an nnz prefix sum.  On a dense band + sparse tail
    the two shards hold (nearly) equal edge counts -- very unequal row counts -- each rank holds
    only its edges, x rows and support rows, and the world-2 step equals the world-1 step."""
    one = _run(1, 300, "mse", tmp_path, skew=True, mode=mode)
    two = _run(2, 300, "mse", tmp_path, skew=True, mode=mode)
    held = two["held"]
    nnz0, nnz1 = int(held[0, 0]), int(held[1, 0])
    rows0, rows1 = int(held[0, 1]), int(held[1, 1])
    assert nnz0 + nnz1 == int(one["held"][0, 0])
    assert abs(nnz0 - nnz1) <= 0.02 * (nnz0 + nnz1), (nnz0, nnz1)
    assert rows0 + rows1 == 300 and rows0 < rows1 / 2, (rows0, rows1)     # balance is by edges, not rows
    s0, s1 = int(held[0, 3]), int(held[1, 3])
    assert abs(s0 - s1) <= 0.05 * (s0 + s1), (s0, s1)                       # support entries balanced too
    _close(one, two)


def test_partition_rows_prefix_sum():
    for p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    from hicgat.dist import ShardPlan, partition_rows, tri_row
    rp = np.concatenate([[0], np.cumsum([100] * 10 + [1] * 90)])     # 10 heavy rows, 90 light ones
    b = partition_rows(rp, 2)
    assert b[0] == 0 and b[2] == 100 and 5 <= b[1] <= 6
    nb = 157
    t = 0
    for I in range(nb):
        for J in range(I, nb):
            if J in (I, nb - 1):
                assert tri_row(t, nb) == I
            t += 1
    # local CSR of a plan: edges of own rows only, columns in buffer numbering
    rowptr = np.array([0, 2, 4, 6, 8])
    col = np.array([0, 1, 0, 1, 2, 3, 2, 3])
    plan = ShardPlan(rowptr, col, 2)
    rp0, c0 = plan.local_csr(0)
    rp1, c1 = plan.local_csr(1)
    assert plan.R == 2 and list(plan.gidx) == [0, 1, 2, 3]
    assert list(rp0) == [0, 2, 4, 4, 4] and list(c0) == [0, 1, 0, 1]
    assert list(rp1) == [0, 0, 0, 2, 4] and list(c1) == [2, 3, 2, 3]
