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
    masks = {n: torch.zeros(p.shape, dtype=torch.bool, device=p.device) for n, p in model.named_parameters()}
    counts = {}
    o = out_pre.detach().double()
    k0 = o.abs() <= margin * o.abs().max()
    counts["conv"] = int(k0.sum())
    cols = k0.any(0)
    masks["conv.bias"] |= cols.to(masks["conv.bias"].device)
    masks["conv.lin_l.weight"] |= cols.to(masks["conv.lin_l.weight"].device)[:, None]
    for (dense, norm), z in zip(BLOCKS, tail_preacts(model, torch.relu(o))):
        k = z.abs() <= margin * z.abs().max()
        counts[norm] = int(k.sum())
        cols = k.any(0)
        for name in (f"{dense}.bias", f"{norm}.weight", f"{norm}.bias"):
            masks[name] |= cols.to(masks[name].device)
        masks[f"{dense}.weight"] |= cols.to(masks[f"{dense}.weight"].device)[:, None]
    return masks, counts


def compare_flat(model, offsets_params, g_ref, g_test, masks=None, skip=("dense3.bias",)):
    """Per parameter (max |diff| over unmasked entries, max |ref| over all, masked count) between two
    flat gradient buffers in FlatAdam layout (``offsets_params`` = zip(opt.params, opt.offsets))."""
    names = {id(p): n for n, p in model.named_parameters()}
    out = {}
    for p, o in offsets_params:
        n = names[id(p)]
        if n in skip:
            continue
        a = g_ref[o:o + p.numel()].view(p.shape).double()
        b = g_test[o:o + p.numel()].view(p.shape).double().to(a.device)
        m = masks[n].to(a.device) if masks is not None else torch.zeros(p.shape, dtype=torch.bool, device=a.device)
        d = (a - b).abs().masked_fill(m, 0.0)
        out[n] = (float(d.max()), float(a.abs().max()), int(m.sum()))
    return out
