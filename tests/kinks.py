"""Kink-aware gradient comparison for two fp32 evaluations of the flagship's training step.

GATNetSelectiveResidualsUpdated (models.py:634-662) has four relus: after the GATConv and after
the three LayerNorms.  Two correct fp32 evaluations that sum in different orders (h-first vs the
aggregate-first GATConv, one GPU vs P shards, the per-layer tail vs the one-kernel tail) agree to
~1e-7 relative, so a relu input closer to 0 than that can fall on either side of the kink, and that
ONE element's gradient then differs by its whole value -- a discontinuity of the reference's own
arithmetic (n = 777: one block-2 LN output at |z| = 6e-8, profiles/r03_relu_margin.txt).

``kink_masks`` finds, in float64, every relu input within ``margin`` x its layer's max |.| of 0
(the rule of tests/test_gpu_fullsize.py's fp64 check: relu decisions of two evaluations differ only
below 1e-6 of the max) and masks the gradient entries such an element decides outright:

* GATConv relu at (row r, column c): ``conv.bias[c]`` and row c of ``conv.lin_l.weight`` (the
  flipped dout[r, c] enters dW only through row c, and db[c]);
* LayerNorm k's relu at (r, c): row c of the block's dense weight, its bias[c], and the LN's
  weight[c] / bias[c].
Everything else -- including the spread-out effect of a flip on upstream gradients (a rank-1
term of ONE row out of N) -- stays inside the ordinary 1e-4-of-max bound, unmasked.

``margin`` 1e-6 and not 1e-5: at N = 20000 a 1e-5 margin holds ~400 LN elements (z ~ N(0, 1) over
9 M relu inputs), which would mask nearly every row of ``densea`` and hide what the test is for;
1e-6 is still ~50x the fp32 disagreement of two orders.
"""
import torch

BLOCKS = (("densea", "norm_a"), ("dense1", "norm1"), ("dense2", "norm2"))


def tail_preacts(model, o):
    """float64 LayerNorm outputs (the relu inputs) of the three tail blocks for tail input ``o``."""
    d = torch.float64
    x = o.detach().to(d)

    def lin(layer, v):
        return v @ layer.weight.detach().to(d).t() + layer.bias.detach().to(d)

    def ln(norm, v):
        return torch.nn.functional.layer_norm(v, v.shape[1:], norm.weight.detach().to(d), norm.bias.detach().to(d),
                                              norm.eps)

    z1 = ln(model.norm_a, lin(model.densea, x))
    x1 = torch.relu(z1) + lin(model.align_densea, x)
    z2 = ln(model.norm1, lin(model.dense1, x1))
    x2 = torch.relu(z2) + lin(model.align_dense1, x1)
    z3 = ln(model.norm2, lin(model.dense2, x2))
    return z1, z2, z3


def kink_masks(model, out_pre, margin=1e-6):
    """(masks, counts): masks = {parameter name: bool tensor (True = decided by a kink)}, counts =
    kink elements per relu.  ``out_pre`` = the GATConv output before its relu (bias included), from
    the model's CURRENT weights (the step being compared)."""
    masks, counts, _ = _kinks(model, out_pre, margin)
    return masks, counts


def _kinks(model, out_pre, margin):
    masks = {n: torch.zeros(p.shape, dtype=torch.bool, device=p.device) for n, p in model.named_parameters()}
    counts, where = {}, {}
    o = out_pre.detach().double()
    k0 = o.abs() <= margin * o.abs().max()
    counts["conv"] = int(k0.sum())
    where["conv"] = k0.nonzero()
    cols = k0.any(0)
    masks["conv.bias"] |= cols.to(masks["conv.bias"].device)
    masks["conv.lin_l.weight"] |= cols.to(masks["conv.lin_l.weight"].device)[:, None]
    for (dense, norm), z in zip(BLOCKS, tail_preacts(model, torch.relu(o))):
        k = z.abs() <= margin * z.abs().max()
        counts[norm] = int(k.sum())
        where[norm] = k.nonzero()
        cols = k.any(0)
        for name in (f"{dense}.bias", f"{norm}.weight", f"{norm}.bias"):
            masks[name] |= cols.to(masks[name].device)
        masks[f"{dense}.weight"] |= cols.to(masks[f"{dense}.weight"].device)[:, None]
    return masks, counts, where


def _relu_grads(model, out_pre, dcoords):
    """float64 autograd of the tail from the GATConv's relu output to the coordinates, seeded with
    the loss gradient ``dcoords``: the gradients at the four relu OUTPUTS (g0 for the GATConv's, g1..g3
    for the LayerNorm blocks'), each block's input, its pre-LN output's 1/sigma and x-hat."""
    d = torch.float64

    def lin(layer, v):
        return v @ layer.weight.detach().to(d).t() + layer.bias.detach().to(d)

    def ln(norm, v):
        mu = v.mean(1, keepdim=True)
        rstd = torch.rsqrt(((v - mu) ** 2).mean(1, keepdim=True) + norm.eps)
        xh = (v - mu) * rstd
        return xh * norm.weight.detach().to(d) + norm.bias.detach().to(d), rstd, xh

    m = model
    o = torch.relu(out_pre.detach().to(d)).requires_grad_(True)
    ins, rs, xhs, outs = [], [], [], []
    v = o
    for dense, norm, align in (("densea", "norm_a", "align_densea"), ("dense1", "norm1", "align_dense1"),
                               ("dense2", "norm2", None)):
        ins.append(v.detach())
        z, rstd, xh = ln(getattr(m, norm), lin(getattr(m, dense), v))
        r = torch.relu(z)
        r.retain_grad()
        outs.append(r)
        rs.append(rstd.detach())
        xhs.append(xh.detach())
        v = r + lin(getattr(m, align), v) if align else r
    coords = lin(m.dense3, v)
    coords.backward(dcoords.detach().to(d))
    return [o.grad] + [r.grad for r in outs], ins, rs, xhs


def kink_bounds(model, out_pre, dcoords, x, rowptr, col, margin=1e-6, slack=2.0):
    """(masks, counts, bounds): ``kink_masks`` plus, for every masked gradient entry, the size of the
    term the flipped relu decides (float64; ``bounds[name]`` has the parameter's shape, 0 where nothing
    flips), so a comparison can CHECK a masked entry -- |diff| <= slack x (sum of its flipped terms) +
    the ordinary bound -- instead of skipping it.  ``dcoords`` = the loss gradient of the coordinates at
    the compared step; ``x``, ``rowptr``, ``col`` = the GATConv input and its CSR (self loops included).

    The flipped term of a relu at (r, c), with g = d loss / d relu-output[r, c] (from ``_relu_grads``):
    * GATConv: dout[r, c] = g or 0.  conv.bias[c] moves by |g|; lin_l.weight[c, k] by |g| |xa_r[k]|,
      xa_r = sum_j alpha_rj x_j a convex combination over r's neighbours, so |xa_r[k]| <= max_j |x_j[k]|;
    * LayerNorm block: dz[r, c] = g or 0, and the LN backward turns it into dy[r, c] = gamma_c / sigma_r
      g (1 - 1/W - xh_c^2 / W); dense.weight[c, k] moves by |gamma_c g / sigma_r| |x_in[r, k]|,
      dense.bias[c] by |gamma_c g / sigma_r|, norm.weight[c] by |g xh[r, c]|, norm.bias[c] by |g|.
    ``slack`` covers the rank-1 side effects of the same flip (the LN row mixing, the attention
    terms), which the unmasked entries already absorb in the 1e-4-of-max bound."""
    masks, counts, where = _kinks(model, out_pre, margin)
    bounds = {n: torch.zeros(p.shape, dtype=torch.float64, device=p.device) for n, p in model.named_parameters()}
    if not any(counts.values()):
        return masks, counts, bounds
    gs, ins, rs, xhs = _relu_grads(model, out_pre, dcoords)
    rp = rowptr.detach().cpu().long()
    cl = col.detach().to(x.device).long()
    xd = x.detach().to(torch.float64)
    W = bounds["conv.lin_l.weight"]
    for r, c in where["conv"].tolist():
        g = float(gs[0][r, c].abs())
        nb = cl[int(rp[r]):int(rp[r + 1])]
        xm = xd[nb].abs().max(0).values
        W[c] += slack * g * xm.to(W.device)
        bounds["conv.bias"][c] += slack * g
    for b, ((dense, norm), key) in enumerate(zip(BLOCKS, ("norm_a", "norm1", "norm2"))):
        gam = getattr(model, norm).weight.detach().to(torch.float64)
        for r, c in where[key].tolist():
            g = float(gs[b + 1][r, c].abs())
            dy = g * abs(float(gam[c])) * float(rs[b][r, 0])
            bounds[f"{dense}.weight"][c] += slack * dy * ins[b][r].abs().to(bounds[f"{dense}.weight"].device)
            bounds[f"{dense}.bias"][c] += slack * dy
            bounds[f"{norm}.weight"][c] += slack * g * abs(float(xhs[b][r, c]))
            bounds[f"{norm}.bias"][c] += slack * g
    return masks, counts, bounds


MAX_MASKED_FRAC = 0.10   # a comparison in which kinks decide more than this share of a tensor says little


def compare_flat(model, offsets_params, g_ref, g_test, masks=None, skip=("dense3.bias",), bounds=None):
    """Per parameter (max excess, max |ref| over all, masked count) between two flat gradient buffers
    in FlatAdam layout (``offsets_params`` = zip(opt.params, opt.offsets)).  The excess is |diff| on
    unmasked entries; on masked entries it is |diff| minus the flipped term's size (``bounds``, from
    ``kink_bounds``: every entry checked), or 0 when no bounds are given (skipped).  Asserts that at
    most MAX_MASKED_FRAC of any tensor is masked."""
    names = {id(p): n for n, p in model.named_parameters()}
    out = {}
    for p, o in offsets_params:
        n = names[id(p)]
        if n in skip:
            continue
        a = g_ref[o:o + p.numel()].view(p.shape).double()
        b = g_test[o:o + p.numel()].view(p.shape).double().to(a.device)
        m = masks[n].to(a.device) if masks is not None else torch.zeros(p.shape, dtype=torch.bool, device=a.device)
        d = (a - b).abs()
        if bounds is not None:
            d = torch.where(m, (d - bounds[n].to(a.device)).clamp_min(0.0), d)
        else:
            d = d.masked_fill(m, 0.0)
        frac = float(m.sum()) / m.numel()
        assert frac <= MAX_MASKED_FRAC, f"{n}: {int(m.sum())} of {m.numel()} gradient entries ({frac:.1%}) decided by kinks"
        out[n] = (float(d.max()), float(a.abs().max()), int(m.sum()))
    return out
