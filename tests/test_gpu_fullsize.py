"""GPU parity at BASELINE.json's full sizes (configs[1] synth-2000 dense, configs[2] synth-20000).

* ``test_synth20000_gat_backward_matches_fp64``: the whole GATConv training-form forward and
  backward (a4, a5, a10: ``agg_fwd_act`` -> ``agg_bwd_rows`` -> ``agg_bwd_src`` -> ``param_grad``)
  on the N = 20000 / 1 % graph (4.0 M edges) against an fp64 evaluation of the same autograd
  (models.py:634-662; PyG 1.7.2 softmax / segment_csr backward) computed
  edge-chunk by edge-chunk with plain torch fp64 ops.  Every row of out, dout, delta, da_dst, dh,
  da_src and all of datt_l, datt_r, dbias are compared, not samples.
* ``test_synth2000_dense_training_step_matches_oracle``: one full training step (forward + MSE +
  backward + Adam) of the flagship model on the dense 2000-node graph (4.0 M edges) against the CPU
  oracle (exact-formula cdist) from the same seed: loss, coordinates, every gradient, every
  parameter after Adam.

Tolerances: forward values 1e-5 relative (the north star's bar); gradients 1e-4 of the tensor's max
magnitude (fp32 reassociation over ~200 - 2000 term sums; the same bound as tests/test_gpu_parity).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import hicgat  # noqa: F401  (fails loudly if libhicgat.so is missing)


def _rel(a, b):
    a = a.double()
    b = b.double().to(a.device)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _fp64_gat_train(rowptr, col, h, att_l, att_r, bias, g, mask, ns=0.2, chunk=1 << 18):
    """fp64 autograd of y = relu(GATConv_agg(h)) for the upstream gradient g (all rows), with the
    relu mask given (the kernel's own fp32 decision; the caller checks it against the fp64 sign):
    returns out (pre-relu, with bias), dout, delta, da_dst, dh (incl. the logit terms), da_src,
    datt_l, datt_r, dbias -- the chain rule written out over the CSR, edge chunk by edge chunk."""
    n, D = h.shape
    H = att_l.shape[-2]
    C = D // H
    h = h.double()
    al, ar = att_l.double().reshape(H, C), att_r.double().reshape(H, C)
    hv = h.view(n, H, C)
    a_s = (hv * al).sum(-1)
    a_d = (hv * ar).sum(-1)
    rp = rowptr.long()
    cl = col.long()
    rows = torch.repeat_interleave(torch.arange(n, device=h.device), rp[1:] - rp[:-1])
    pre = a_s[cl] + a_d[rows]                                              # [E, H]
    e = torch.nn.functional.leaky_relu(pre, ns)
    emax = torch.full((n, H), float("-inf"), dtype=torch.float64, device=h.device).scatter_reduce(
        0, rows.view(-1, 1).expand_as(e), e, reduce="amax", include_self=True)
    u = (e - emax[rows]).exp()
    usum = torch.zeros((n, H), dtype=torch.float64, device=h.device).index_add(0, rows, u)
    alpha = u / (usum[rows] + 1e-16)
    slope = torch.where(pre > 0, 1.0, ns).double()
    E = cl.numel()
    agg = torch.zeros((n, H, C), dtype=torch.float64, device=h.device)
    for s in range(0, E, chunk):
        sl = slice(s, min(E, s + chunk))
        agg.index_add_(0, rows[sl], hv[cl[sl]] * alpha[sl].unsqueeze(-1))
    out = agg.reshape(n, D) + bias.double()
    dout = torch.where(mask, g.double(), torch.zeros_like(out))
    dv = dout.view(n, H, C)
    gij = torch.empty((E, H), dtype=torch.float64, device=h.device)
    for s in range(0, E, chunk):
        sl = slice(s, min(E, s + chunk))
        gij[sl] = (dv[rows[sl]] * hv[cl[sl]]).sum(-1)
    delta = torch.zeros((n, H), dtype=torch.float64, device=h.device).index_add(0, rows, alpha * gij)
    ds = alpha * (gij - delta[rows]) * slope
    da_dst = torch.zeros((n, H), dtype=torch.float64, device=h.device).index_add(0, rows, ds)
    da_src = torch.zeros((n, H), dtype=torch.float64, device=h.device).index_add(0, cl, ds)
    dh = torch.zeros((n, H, C), dtype=torch.float64, device=h.device)
    for s in range(0, E, chunk):
        sl = slice(s, min(E, s + chunk))
        dh.index_add_(0, cl[sl], dv[rows[sl]] * alpha[sl].unsqueeze(-1))
    dh += da_src.unsqueeze(-1) * al + da_dst.unsqueeze(-1) * ar
    datt_l = (da_src.unsqueeze(-1) * hv).sum(0).reshape(-1)
    datt_r = (da_dst.unsqueeze(-1) * hv).sum(0).reshape(-1)
    return dict(out=out, dout=dout, delta=delta, da_dst=da_dst, dh=dh.reshape(n, D), da_src=da_src,
                datt_l=datt_l, datt_r=datt_r, dbias=dout.sum(0), a_s=a_s, a_d=a_d)


@pytest.mark.parametrize("tiled", [False, True], ids=["gather", "tiled"])
def test_synth20000_gat_backward_matches_fp64(tiled):
    """tiled: the dense 32x32 tiles on the matrix cores (hicgat_gat_agg_fwd_tiled /
    hicgat_gat_agg_bwd_src_tiled, default HICGAT_TILE_MIN), the rest gathered."""
    import hicgat
    from hicgat import synth
    K = hicgat.kernels.default()
    n = 20000
    i, j, c = synth.contact_pairs(n, density=0.01, seed=0)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    del A
    torch.manual_seed(0)
    conv = hicgat.GATConv(512, 256, heads=2).to(DEV)
    x = torch.tensor(synth.features(n), device=DEV)
    with torch.no_grad():
        conv.bias.copy_(0.05 * torch.randn_like(conv.bias))     # relu mask not trivially all-on
        att_l, att_r, bias = conv.att_l.detach(), conv.att_r.detach(), conv.bias.detach()
        h, a_s, a_d = K.linear_att(x, conv.lin_l.weight.detach(), att_l, att_r)
    g = torch.randn(n, 512, device=DEV)
    out = torch.empty(n, 512, device=DEV)
    out2 = torch.empty(n, 512, device=DEV)
    rs = torch.empty(n, 8, device=DEV)
    tiles = hicgat.graph.build_tiles(adj.rowptr32, adj.col32, 0, n, n, 64) if tiled else None
    if tiled:
        assert tiles.n_dense > 0.4 * adj.device_nnz
        K.agg_fwd_tiled(adj.rowptr32, adj.col32, tiles, h, a_s, a_d, bias, 0.2, 1, out, out2, rs)
    else:
        K.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, bias, 0.2, 1, out, out2, rs)
    dout = torch.empty(n, 512, device=DEV)
    K.agg_bwd_rows(0, n, 1, g, out, bias, out2, dout, rs)
    dh = torch.empty(n, 512, device=DEV)
    da_src = torch.empty(n, 2, device=DEV)
    if tiled:
        K.agg_bwd_src_tiled(tiles, h, a_s, a_d, rs, dout, att_l, att_r, 0.2, dh, da_src)
    else:
        K.agg_bwd_src(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, rs, dout, att_l, att_r, 0.2, dh, da_src)
    datt_l, datt_r, dbias = K.param_grad(h, dout, da_src, rs, 2)
    # any subset of the three parts (the split the training backward issues: datt_dst + dbias
    # beside the source pass, datt_src behind it) is bitwise the all-parts call
    parts = [torch.full((512,), 7.0, device=DEV) for _ in range(3)]
    K.param_grad(h, dout, None, rs, 2, out=(None, parts[1], parts[2]))
    K.param_grad(h, None, da_src, rs, 2, out=(parts[0], None, None))
    torch.cuda.synchronize()
    for got, want in zip(parts, (datt_l, datt_r, dbias)):
        assert torch.equal(got, want)
    ref = _fp64_gat_train(adj.rowptr32, adj.col32, h, att_l, att_r, bias, g, out > 0)
    # relu decisions may differ from fp64 only where the pre-activation is at rounding level
    flip = (out > 0) != (ref["out"] > 0)
    assert float(ref["out"][flip].abs().max()) < 1e-6 * float(ref["out"].abs().max()) if flip.any() else True
    # the logits of the MFMA epilogue vs fp64 of the same h
    assert _rel(a_s, ref["a_s"]) < 1e-5 and _rel(a_d, ref["a_d"]) < 1e-5
    errs = {
        "out": _rel(out, torch.relu(ref["out"])),
        "dout": _rel(dout, ref["dout"]),
        "delta": _rel(rs[:, 4:6], ref["delta"]),
        "da_dst": _rel(rs[:, 6:8], ref["da_dst"]),
        "dh": _rel(dh, ref["dh"]),
        "da_src": _rel(da_src, ref["da_src"]),
        "datt_l": _rel(datt_l, ref["datt_l"]),
        "datt_r": _rel(datt_r, ref["datt_r"]),
        "dbias": _rel(dbias, ref["dbias"]),
    }
    print("max |err| / max |ref|:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert errs["out"] < 1e-5 and errs["dout"] == 0.0, errs
    for k in ("delta", "da_dst", "dh", "da_src", "datt_l", "datt_r", "dbias"):
        assert errs[k] < 1e-4, (k, errs)


@pytest.mark.timeout(600)
def test_synth2000_dense_training_step_matches_oracle():
    import hicgat
    from hicgat import synth
    from oracle import gat as og
    from oracle import graph as ogr
    n = 2000
    i, j, c = synth.contact_pairs(n, density=None, seed=0)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    x = synth.features(n, seed=0)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
    loss, stats, coords = hicgat.train.train_step(model, opt, torch.tensor(x, device=DEV), adj, tr)
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().clone() for k, p in model.named_parameters()}
    params = {k: p.detach().cpu().clone() for k, p in model.named_parameters()}

    # the oracle: same seed, same graph (host CSR of the dense contacts), exact distances
    Ah = A.cpu().numpy()
    d = ogr.load_input(Ah, x)
    t_ref = ogr.cont2dist(d["y"], 0.5).float()
    assert torch.equal(tr.dense().cpu(), t_ref)
    torch.manual_seed(0)
    ref = og.GATNetSelectiveResidualsUpdated()
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        radj = (torch.tensor(d["rowptr"]), torch.tensor(d["col"]))
        c_ref = ref.get_model(d["x"], radj)
        l_ref = torch.nn.functional.mse_loss(torch.cdist(c_ref, c_ref, compute_mode=og.CDIST_MODE).float(), t_ref)
        l_ref.backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    rel_l = abs(loss.item() - l_ref.item()) / l_ref.item()
    rel_c = _rel(coords.detach().cpu(), c_ref.detach())
    print(f"loss {loss.item():.8g} vs oracle {l_ref.item():.8g} (rel {rel_l:.2e}); coords rel {rel_c:.2e}")
    assert rel_l < 1e-5 and rel_c < 1e-5
    gscale = max(p.grad.abs().max().item() for p in ref.parameters())
    worst = {}
    for k, pr in ref.named_parameters():
        if pr.grad.abs().max().item() < 1e-3 * gscale:       # exactly 0 in exact arithmetic (dense3.bias)
            assert grads[k].abs().max().item() < 1e-3 * gscale, k
            continue
        worst[k] = _rel(grads[k], pr.grad)
    print("grad max |err| / max |ref|:", {k: f"{v:.1e}" for k, v in worst.items()})
    assert max(worst.values()) < 2e-4, worst
    ropt.step()
    # Adam's first step moves a parameter by lr * g / (|g| + eps): compare it where that is not
    # sensitive to the gradient's rounding, |g| >> eps = 1e-8 and above 1e-3 of the tensor's max
    # (there d(update)/dg = lr eps / (|g| + eps)^2 keeps the update error below 1e-6)
    for k, pr in ref.named_parameters():
        g_ref = pr.grad
        sig = (g_ref.abs() > 1e-3 * g_ref.abs().max()) & (g_ref.abs() > 1e-6)
        if not sig.any():
            continue
        diff = (params[k] - pr.detach()).abs()
        assert float(diff[sig].max()) < 1e-6, k


def test_synth20000_support_form_loss_matches_dense():
    """configs[2] (N = 20000, 1 % contacts): the fused loss over the truth's background + support
    form (the default for cont2dist's target) against the dense-truth kernel and an fp64
    evaluation on sampled rows: mse / moments 1e-6 relative, dcoords 1e-5 of their max."""
    import hicgat
    from hicgat import synth
    n = 20000
    i, j, c = synth.contact_pairs(n, density=0.01, seed=0)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    del A
    sf = tr.support
    assert sf is not None
    K = hicgat.kernels.default()
    rng = np.random.default_rng(0)
    coords = torch.tensor(rng.standard_normal((n, 3)).astype(np.float32), device=DEV)
    res = {}
    for kind in (0, 1):
        for form in ("dense", "support"):
            stats = torch.empty(12, dtype=torch.float64, device=DEV)
            loss = torch.empty((), dtype=torch.float32, device=DEV)
            dc = torch.empty_like(coords)
            if form == "dense":
                K.fused_loss(coords, tr.buf, n, kind, 0, -1, stats, loss, dc)
            else:
                K.fused_loss_support(coords, sf, n, kind, stats, loss, dc)
            res[kind, form] = (stats.cpu().numpy(), dc)
    for kind in (0, 1):
        sd, gd = res[kind, "dense"]
        ss, gs = res[kind, "support"]
        for k in (0, 6, 7) if kind == 0 else (0, 1, 2, 3, 4, 5, 7):
            assert abs(ss[k] - sd[k]) <= 1e-6 * max(abs(sd[k]), 1e-30), (kind, k, ss[k], sd[k])
        if kind == 1:
            assert abs(ss[8] - sd[8]) < 1e-6
        assert _rel(gs, gd) < 1e-5
    # fp64 gradient of the MSE on 64 sampled rows: dL/dc_i = 4/N^2 sum_j (d_ij - t_ij)/d_ij (c_i - c_j)
    cd = coords.double()
    rows = torch.tensor(rng.choice(n, 64, replace=False), device=DEV)
    diff = cd[rows, None, :] - cd[None, :, :]
    d = diff.norm(dim=-1)
    t = tr.dense()[rows].double()
    w = torch.where(d > 0, (d - t) / d.clamp_min(1e-300), torch.zeros_like(d))
    g_ref = 4.0 / n / n * (w[..., None] * diff).sum(1)
    assert _rel(res[0, "support"][1][rows], g_ref) < 1e-5
    print(f"support nnz {sf.nnz} ({sf.nnz / n / n:.2%}); mse {res[0, 'support'][0][7]:.9g} vs dense "
          f"{res[0, 'dense'][0][7]:.9g}")


@pytest.mark.timeout(900)
def test_synth20000_training_step_matches_oracle():
    """BASELINE configs[2] -- bench.py's headline workload exactly (N = 20000, 1 % power-law contacts,
    seed 0, 4.02 M edges): one whole training step of the flagship (forward, MSE, backward, Adam;
    HiC-GNN_main.py:126-130) on the device against the CPU oracle from the same seed-0 weights
    (exact-formula distances, as the device computes them): loss and coordinates to
    1e-5 relative (the north star's bar), every gradient to 2e-4 of its tensor's max with the entries
    a relu at rounding distance from its kink decides bounded by their flipped term
    (tests/kinks.py::kink_bounds), and the Adam update wherever it does not hinge on the gradient's
    rounding."""
    import hicgat
    from hicgat import synth
    from kinks import compare_flat, kink_bounds
    from oracle import gat as og
    from oracle import graph as ogr
    n = 20000
    i, j, c = synth.contact_pairs(n, density=0.01, seed=0)
    A = synth.dense_contacts(n, i, j, c, device=DEV)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    tr = hicgat.Truth.from_contacts(A, 0.5)
    del A
    xh = synth.features(n, seed=0)
    x = torch.tensor(xh, device=DEV)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(DEV)
    opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
    # kink masks / flipped-term bounds at the step-1 weights (the device's fp32 relu inputs)
    cv = model.conv
    with torch.no_grad():
        out_pre = hicgat.ops.gat_conv(x, cv.lin_l.weight, cv.att_l, cv.att_r, cv.bias, adj)
        c0 = model.get_model(x, adj)
    cd = c0.detach().requires_grad_(True)
    l0, _ = hicgat.ops.fused_dist_loss(cd, tr)
    l0.backward()
    masks, counts, bounds = kink_bounds(model, out_pre, cd.grad, x, adj.rowptr32, adj.col32)
    del out_pre, cd, l0
    loss, _, coords = hicgat.train.train_step(model, opt, x, adj, tr)
    torch.cuda.synchronize()
    loss_d = float(loss.item())
    coords_d = coords.detach().cpu().clone()
    g_dev = opt.grad.detach().clone()
    params = {k: p.detach().cpu().clone() for k, p in model.named_parameters()}

    # the oracle on the host: the CSR of the same pairs (utils.load_input's symmetric, sorted form),
    # cont2dist of the same contacts, the same features and seed
    rows = np.concatenate([i, j])
    cols = np.concatenate([j, i])
    order = np.lexsort((cols, rows))
    rows, cols = rows[order], cols[order]
    rp = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rp, rows + 1, 1)
    radj = (torch.tensor(np.cumsum(rp)), torch.tensor(cols.astype(np.int64)))
    y = torch.zeros((n, n), dtype=torch.float64)
    y[torch.tensor(i), torch.tensor(j)] = torch.tensor(c)
    y[torch.tensor(j), torch.tensor(i)] = torch.tensor(c)
    t_ref = ogr.cont2dist(y, 0.5).float()
    del y
    torch.manual_seed(0)
    ref = og.GATNetSelectiveResidualsUpdated()
    ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        c_ref = ref.get_model(torch.tensor(xh), radj)
        l_ref = torch.nn.functional.mse_loss(torch.cdist(c_ref, c_ref, compute_mode=og.CDIST_MODE).float(), t_ref)
        l_ref.backward()
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"
    rel_l = abs(loss_d - l_ref.item()) / l_ref.item()
    rel_c = _rel(coords_d, c_ref.detach())
    print(f"synth-20000 step 1: loss {loss_d:.9g} vs oracle {l_ref.item():.9g} (rel {rel_l:.2e}); coords rel {rel_c:.2e}; "
          f"kinks {counts}")
    assert rel_l < 1e-5 and rel_c < 1e-5
    # the oracle's gradients in the device's flat layout
    rg = dict(ref.named_parameters())
    names = {id(p): k for k, p in model.named_parameters()}
    g_ref = torch.zeros_like(g_dev)
    for p, o in zip(opt.params, opt.offsets):
        g_ref[o:o + p.numel()] = rg[names[id(p)]].grad.reshape(-1).to(g_ref.device)
    per = compare_flat(model, zip(opt.params, opt.offsets), g_ref, g_dev, masks, bounds=bounds)
    print("grad max excess / max |ref| (masked):", {k: f"{d / m:.1e} ({c_})" for k, (d, m, c_) in per.items()})
    for k, (d, m, _) in per.items():
        assert d <= 2e-4 * m, (k, d, m)
    gscale = max(float(g_ref.abs().max()), 1e-30)
    assert float(rg["dense3.bias"].grad.abs().max()) < 1e-3 * gscale        # 0 in exact arithmetic
    ropt.step()
    for k, pr in ref.named_parameters():
        gr = pr.grad
        sig = (gr.abs() > 1e-3 * gr.abs().max()) & (gr.abs() > 1e-6) & ~masks[k].cpu()
        if sig.any():
            assert float((params[k] - pr.detach()).abs()[sig].max()) < 1e-6, k
