"""GPU: the aggregate-first GATConv kernels (gat_xagg.hip) one by one against the float64 torch
stand-ins of tests/cpu_kernels.py (which tests/test_dist_gloo.py ties to the h-first form and the
autograd oracle), on a 600-node synthetic Hi-C graph sharded over 3 ranks (rank 1's rows)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd"), HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def case():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hicgat
    from hicgat import synth
    from hicgat.dist import ShardPlan
    n = 600
    i, j, c = synth.contact_pairs(n, density=0.05, seed=11)
    A = synth.dense_contacts(n, i, j, c, device="cuda")
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    plan = ShardPlan(adj.rowptr32.cpu().numpy(), adj.col32.cpu().numpy(), 3)
    rank = 1
    r0, r1, _ = plan.rows(rank)
    rp, cl = plan.own_csr(rank)
    srp, scl = plan.slab_csr(rank)
    perm = plan.slab_perm(rank)
    g = torch.Generator().manual_seed(3)
    x = 0.1 * torch.randn((n, 512), generator=g)
    torch.manual_seed(0)
    conv = hicgat.GATConv(512, 256, heads=2)
    W = conv.lin_l.weight.detach().clone()
    al, ar = conv.att_l.detach().clone(), conv.att_r.detach().clone()
    return dict(n=n, r0=r0, r1=r1, rp=torch.from_numpy(rp), cl=torch.from_numpy(cl), srp=torch.from_numpy(srp),
                perm=torch.from_numpy(perm), x=x, W=W, al=al, ar=ar, nnz=int(cl.shape[0]))


def test_xagg_kernels_match_float64_reference(case):
    import hicgat
    from cpu_kernels import CpuKernels
    K, R = hicgat.kernels.default(), CpuKernels()
    d = case
    n, r0, r1 = d["n"], d["r0"], d["r1"]
    rows = r1 - r0
    dev = {k: (v.cuda() if torch.is_tensor(v) else v) for k, v in d.items()}
    out = {}
    for name, kern, t in (("ref", R, d), ("gpu", K, dev)):
        loc = "cuda" if name == "gpu" else "cpu"
        a_src = torch.zeros((n, 2), device=loc)
        a_dst = torch.zeros((n, 2), device=loc)
        kern.xagg_logits(t["x"], t["W"], t["al"], t["ar"], a_src, a_dst)
        out[name] = {"a_src": a_src.clone(), "a_dst": a_dst.clone()}
        if name == "gpu":
            # the rest from the SAME logits (the reference's): each comparison isolates one kernel
            a_src.copy_(out["ref"]["a_src"])
            a_dst.copy_(out["ref"]["a_dst"])
        X4 = torch.zeros((2, 2, rows, 512), device=loc)
        rs = torch.zeros((n, 8), device=loc)
        kern.xagg_fwd(t["rp"], t["cl"], r0, r1, t["x"], a_src, a_dst, 0.2, X4, rs)
        out[name].update(X4=X4.clone(), rs=rs.clone())
        # backward pieces from a fixed upstream gradient
        gen = torch.Generator().manual_seed(7)
        gout = torch.randn((rows, 512), generator=gen).to(loc)
        y0 = torch.randn((rows, 512), generator=gen).to(loc)
        bb = torch.randn(512, generator=gen).to(loc)
        dout = torch.empty((rows, 512), device=loc)
        kern.xagg_rows_bwd(1, gout, y0, bb, dout, rs[r0:r1])
        out[name].update(dout=dout.clone(), rs_rows=rs[r0:r1].clone())
        dxa = torch.randn((rows, 1024), generator=gen).to(loc)
        ds = torch.zeros((d["nnz"], 2), device=loc)
        rs_pre = rs.clone()
        kern.xagg_edge(t["rp"], t["cl"], r0, r1, t["x"], a_src, a_dst, rs, dxa, 0.2, ds, xa2=X4[:, 1])
        # the edge pass with g_src folded in (the sharded step's form): g_src = column sums of its
        # partial rows, da_dst as above
        gpart = torch.zeros((kern.edge_acc_blocks(rows), 1024), device=loc)
        kern.xagg_edge_acc(t["rp"], t["cl"], r0, r1, t["x"], a_src, a_dst, rs_pre, dxa, 0.2, gpart, xa2=X4[:, 1])
        out[name].update(g_src_acc=gpart.double().sum(0), rs_edge_acc=rs_pre[r0:r1].clone())
        da_src = torch.zeros((n, 2), device=loc)
        g_src = torch.zeros(1024, device=loc)
        kern.xagg_slab_sum(t["srp"], t["perm"], ds, t["x"], da_src, g_src)
        out[name].update(ds=ds.clone(), da_src=da_src.clone(), g_src=g_src.clone(), rs_edge=rs[r0:r1].clone())
        gs = torch.randn(1024, generator=gen).to(loc)
        gd = torch.randn(1024, generator=gen).to(loc)
        dW = torch.randn((512, 512), generator=gen).to(loc)
        dl = torch.randn(512, generator=gen).to(loc)
        dr = torch.randn(512, generator=gen).to(loc)
        kern.xagg_param_finish(t["W"], t["al"], t["ar"], gs, gd, dW, dl, dr)
        out[name].update(dW=dW, dl=dl, dr=dr)
        y0 = torch.randn((rows, 512), generator=gen).to(loc)
        o = torch.empty_like(y0)
        kern.xagg_bias_relu(y0, torch.randn(512, generator=gen).to(loc), o)
        out[name].update(y0=y0, o=o)
    g, r = out["gpu"], out["ref"]
    errs = {k: _rel(g[k], r[k]) for k in ("a_src", "a_dst", "X4", "dout", "rs_rows", "ds", "da_src", "g_src",
                                           "rs_edge", "dW", "dl", "dr", "y0", "o", "g_src_acc", "rs_edge_acc")}
    errs["g_src_acc_vs_slab"] = _rel(g["g_src_acc"], r["g_src"])
    errs["rs_stats"] = _rel(g["rs"][d["r0"]:d["r1"], :4], r["rs"][d["r0"]:d["r1"], :4])
    errs["rs_s3"] = _rel(g["rs"][d["r0"]:d["r1"], 4:6], r["rs"][d["r0"]:d["r1"], 4:6])
    print({k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < 1e-5 for v in errs.values()), errs


@pytest.mark.parametrize("shape", ["fwd_1554", "dxa_777", "dw_777_split"])
def test_xagg_gemm_calls_match_float64(shape):
    """The GEMM calls of the xagg step (hicgat.dist._step_xagg) at the world-1 n = 777 shapes, with
    their strided operands and outputs, against float64 torch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hicgat
    from hicgat import ops
    K = hicgat.kernels.default()
    g = torch.Generator().manual_seed(5)
    R = 777
    W = torch.randn((512, 512), generator=g).cuda()
    if shape == "fwd_1554":
        X4 = torch.randn((2, 2, R, 512), generator=g).cuda()
        Y2 = torch.zeros((2, R, 512)).cuda()
        Y2f = Y2.view(2 * R, 512)
        for hd in range(2):
            K.gemm(0, 0, 2 * R, 256, 512, X4[hd].view(2 * R, 512), W[hd * 256:(hd + 1) * 256], Y2f[:, hd * 256:(hd + 1) * 256])
        ref = torch.cat([X4[hd].view(2 * R, 512).double() @ W[hd * 256:(hd + 1) * 256].double().t() for hd in range(2)], 1)
        got = Y2f
    elif shape == "dxa_777":
        dout = torch.randn((R, 512), generator=g).cuda()
        dxa = torch.zeros((R, 1024)).cuda()
        for hd in range(2):
            K.gemm(0, 1, R, 512, 256, dout[:, hd * 256:(hd + 1) * 256], W[hd * 256:(hd + 1) * 256], dxa[:, hd * 512:(hd + 1) * 512])
        ref = torch.cat([dout[:, hd * 256:(hd + 1) * 256].double() @ W[hd * 256:(hd + 1) * 256].double() for hd in range(2)], 1)
        got = dxa
    else:
        dout = torch.randn((R, 512), generator=g).cuda()
        X4 = torch.randn((2, 2, R, 512), generator=g).cuda()
        dW = torch.randn((512, 512), generator=g).cuda()
        ref = dW.double().clone()
        for hd in range(2):
            K.gemm(1, 1, 256, 512, R, dout[:, hd * 256:(hd + 1) * 256], X4[hd, 0], dW[hd * 256:(hd + 1) * 256],
                   accumulate=True, splits=ops._splits(256, 512, R))
            ref[hd * 256:(hd + 1) * 256] += dout[:, hd * 256:(hd + 1) * 256].double().t() @ X4[hd, 0].double()
        got = dW
    err = _rel(got, ref)
    print(shape, f"{err:.2e}")
    assert err < 1e-5


@pytest.mark.parametrize("target", [64, 512])
def test_param_grads_grouped_matches_float64(target):
    """hicgat_param_grads_grouped (the sharded step's one-launch parameter gradients) against
    float64 torch: weight-gradient jobs of the step's shapes -- a 512 x 512 dual-Linear pair with
    its bias, the two per-head 256 x 512 blocks of lin_l (row views of one [512, 512] gradient) with
    their bias halves, dense3's 3 x 64 (scalar-staged tile), g_dst's 2 x 512 from a strided [R, 8]
    row-stats view (overwrite) -- and column-sum jobs (LayerNorm partial rows into an adjacent
    [dgamma | dbeta], a [blocks, 1024] partial-row sum that overwrites); ``target`` = the workgroup
    budget (64: few K chunks, 512: many).  Then the same call again must give the same bits."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hicgat
    K = hicgat.kernels.default()
    g = torch.Generator().manual_seed(9)
    R = 2517

    def rnd(*shape):
        return torch.randn(shape, generator=g).cuda()

    x, dY, dout, z3, dc, rs = rnd(R, 512), rnd(R, 512), rnd(R, 512), rnd(R, 64), rnd(R, 3), rnd(R, 8)
    Wg, bg, W3g, b3g = rnd(512, 512), rnd(512), rnd(3, 64), rnd(3)
    Wl, bl = rnd(512, 512), rnd(512)
    gdst = rnd(2, 512)
    lnp, lng = rnd(633, 512), rnd(512)
    gp, gs = rnd(512, 1024), rnd(1024)
    ref = {"Wg": Wg.double() + dY.double().t() @ x.double(), "bg": bg.double() + dY.double().sum(0),
           "W3g": W3g.double() + dc.double().t() @ z3.double(), "b3g": b3g.double() + dc.double().sum(0),
           "gdst": rs[:, 6:8].double().t() @ x.double(), "lng": lng.double() + lnp.double().sum(0),
           "gs": gp.double().sum(0)}
    Wl_ref, bl_ref = Wl.double().clone(), bl.double().clone()
    for hd in range(2):
        sl = slice(hd * 256, (hd + 1) * 256)
        Wl_ref[sl] += dout[:, sl].double().t() @ x.double()
        bl_ref[sl] += dout[:, sl].double().sum(0)
    ref.update(Wl=Wl_ref, bl=bl_ref)
    outs = {"Wg": Wg, "bg": bg, "W3g": W3g, "b3g": b3g, "gdst": gdst, "lng": lng, "gs": gs, "Wl": Wl, "bl": bl}
    init = {k: v.clone() for k, v in outs.items()}
    res = []
    for rep in range(2):
        for k in outs:
            outs[k].copy_(init[k])
        w = [(dY, x, Wg, bg, True), (dc, z3, W3g, b3g, True), (rs[:, 6:8], x, gdst, None, False)]
        w += [(dout[:, hd * 256:(hd + 1) * 256], x, Wl[hd * 256:(hd + 1) * 256], bl[hd * 256:(hd + 1) * 256], True)
              for hd in range(2)]
        K.param_grads_grouped(w, [(lnp, lng, True), (gp, gs, False)], target_wgs=target)
        torch.cuda.synchronize()
        res.append({k: v.clone() for k, v in outs.items()})
    errs = {k: _rel(res[0][k], ref[k]) for k in ref}
    print(target, {k: f"{v:.1e}" for k, v in errs.items()})
    assert all(v < 1e-5 for v in errs.values()), errs
    assert all(torch.equal(res[0][k], res[1][k]) for k in outs)


@pytest.mark.parametrize("n,world", [(3000, 2), (20000, 8)])
def test_xagg_side_branch_equals_serial_order_with_a_real_reduce(n, world):
    """The xagg step runs its side branch (grouped dW, then the all-reduce of the WHOLE flat
    gradient) on the "grad" stream while the edge pass, g's column sums and g's all-reduce run on the
    step's stream.  That is correct only if nothing on the step's stream touches opt.grad between the
    fork and the join.  A communicator whose all-reduce really changes its buffer in place on the
    issuing stream (t *= P, as a sum over P equal ranks would) makes any such race visible: the
    captured overlapped step must replay bit-equal to the same launches in serial order
    (dist.XAGG_SIDE_BRANCH = False), gradients and parameters, over three replays."""
    for p in (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),):
        if p not in sys.path:
            sys.path.insert(0, p)
    import hicgat
    from hicgat import dist as hdist
    from hicgat import synth

    class ScaleComm(hdist.SimComm):
        def __init__(self, P, rank):
            super().__init__(P, rank, emulate=False)

        def all_reduce(self, t, name="all_reduce"):
            t.mul_(float(self.P))

    density, seed = (0.01, 0) if n == 20000 else (0.05, 3)
    i, j, c = synth.contact_pairs(n, density=density, seed=seed)
    A = synth.dense_contacts(n, i, j, c, device="cuda")
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    truth = hicgat.Truth.from_contacts(A, 0.5)
    del A
    x = torch.tensor(synth.features(n, seed=seed), device="cuda")
    res = {}
    saved = hdist.XAGG_SIDE_BRANCH
    try:
        for side in (False, True):
            hdist.XAGG_SIDE_BRANCH = side
            torch.manual_seed(0)
            model = hicgat.GATNetSelectiveResidualsUpdated().to("cuda")
            tr = hdist.ShardedTrainer(model, x, adj, truth, lr=1e-3, mode="xagg", comm=ScaleComm(world, 0))
            step = tr.captured(warmup=1)
            out = []
            for _ in range(3):
                loss = float(step()[0])
                out.append((loss, tr.opt.grad.clone(), tr.opt.flat.clone()))
            torch.cuda.synchronize()
            res[side] = out
            del step, tr, model
    finally:
        hdist.XAGG_SIDE_BRANCH = saved
    for (l0, g0, p0), (l1, g1, p1) in zip(res[False], res[True]):
        assert l0 == l1 and torch.equal(g0, g1) and torch.equal(p0, p1)


@pytest.mark.parametrize("n,world", [(3000, 2), (20000, 8)])
def test_xagg_step_pack_in_first_launch_is_bitwise(monkeypatch, n, world):
    """The head-fused tail's packed weights (W1c, W2c and lin_l's W) written by the xagg step's first
    launch (hicgat_xagg_logits_zero_pack) against the tail forward's own hicgat_tail_pack launch
    (ops.STEP_PACK = False): the captured step replays to the same loss, gradients and parameters bit
    for bit, and after each replay the buffer holds exactly the pack of that step's weights."""
    for p in (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),):
        if p not in sys.path:
            sys.path.insert(0, p)
    import hicgat
    from hicgat import dist as hdist
    from hicgat import kernels, ops, synth
    density, seed = (0.01, 0) if n == 20000 else (0.05, 3)
    i, j, c = synth.contact_pairs(n, density=density, seed=seed)
    A = synth.dense_contacts(n, i, j, c, device="cuda")
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    truth = hicgat.Truth.from_contacts(A, 0.5)
    del A
    x = torch.tensor(synth.features(n, seed=seed), device="cuda")
    res = {}
    for fold in (False, True):
        monkeypatch.setattr(ops, "STEP_PACK", fold)
        torch.manual_seed(0)
        model = hicgat.GATNetSelectiveResidualsUpdated().to("cuda")
        tr = hdist.ShardedTrainer(model, x, adj, truth, lr=1e-3, mode="xagg", comm=hdist.SimComm(world, 0))
        step = tr.captured(warmup=1)
        out = []
        for _ in range(3):
            m = model
            W1c = torch.cat([m.densea.weight, m.align_densea.weight]).detach()
            W2c = torch.cat([m.dense1.weight, m.align_dense1.weight]).detach()
            want = kernels.default().tail_pack(W1c, W2c, m.conv.lin_l.weight.detach().contiguous())
            loss = float(step()[0])
            torch.cuda.synchronize()
            if fold:
                assert torch.equal(model._hicgat_pack_buf, want)
            out.append((loss, tr.opt.grad.clone(), tr.opt.flat.clone()))
        res[fold] = out
        del step, tr, model
    for (l0, g0, p0), (l1, g1, p1) in zip(res[False], res[True]):
        assert l0 == l1 and torch.equal(g0, g1) and torch.equal(p0, p1)
