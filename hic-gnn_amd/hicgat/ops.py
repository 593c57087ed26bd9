"""Autograd functions over the HIP kernels (the product compute path; no CPU fallback).

* ``gat_conv``        -- PyG 1.7.2 GATConv forward/backward (a2, a4, a5 and their backward).
* ``pairwise_dist``   -- torch.cdist(c, c, p=2) forward/backward (a7), D materialised.
* ``fused_dist_loss`` -- cdist + MSELoss (+ Pearson / combined loss value) fused (a7-a9), D never
                         materialised; returns the loss scalar and keeps the fp64 stats.
"""
import torch

from . import _lib

# Optional live kernel timing (bench.py): name -> list of (start, end) torch.cuda.Event pairs,
# recorded on the stream each kernel is launched on.
TIMERS = None


class _timed:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if TIMERS is not None:
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e0.record()

    def __exit__(self, *a):
        if TIMERS is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            TIMERS.setdefault(self.name, []).append((self.e0, e1))


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.HicgatUnavailable("hicgat ops need CUDA (HIP) tensors; got a CPU tensor")


class _GATConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, att_l, att_r, bias, rowptr, col, negative_slope):
        lib = _lib.lib()
        _dev_check(x, W, att_l, att_r, bias, rowptr, col)
        x = x.contiguous()
        W = W.contiguous()
        N, F = x.shape
        H, C = att_l.shape[-2], att_l.shape[-1]
        D = H * C
        dev = x.device
        s = _lib.stream(dev)
        h = torch.empty((N, D), dtype=torch.float32, device=dev)
        a_src = torch.empty((N, H), dtype=torch.float32, device=dev)
        a_dst = torch.empty_like(a_src)
        al = att_l.contiguous()
        ar = att_r.contiguous()
        with _timed("gat_linear_att"):
            _lib.check(lib.hicgat_gat_linear_att(_lib.ptr(x), _lib.ptr(W), _lib.ptr(al), _lib.ptr(ar), N, F,
                                                 H, C, _lib.ptr(h), _lib.ptr(a_src), _lib.ptr(a_dst), s),
                       "hicgat_gat_linear_att")
        b = bias if bias is not None else torch.zeros(D, dtype=torch.float32, device=dev)
        out = torch.empty((N, D), dtype=torch.float32, device=dev)
        rmax = torch.empty((N, H), dtype=torch.float32, device=dev)
        rsum = torch.empty_like(rmax)
        with _timed("gat_agg_fwd"):
            _lib.check(lib.hicgat_gat_agg_fwd(_lib.ptr(rowptr), _lib.ptr(col), N, col.numel(), H, C,
                                              _lib.ptr(h), _lib.ptr(a_src), _lib.ptr(a_dst), _lib.ptr(b),
                                              float(negative_slope), _lib.ptr(out), _lib.ptr(rmax),
                                              _lib.ptr(rsum), s), "hicgat_gat_agg_fwd")
        ctx.save_for_backward(x, W, al, ar, h, a_src, a_dst, rmax, rsum, rowptr, col)
        ctx.has_bias = bias is not None
        ctx.ns = float(negative_slope)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = _lib.lib()
        x, W, al, ar, h, a_src, a_dst, rmax, rsum, rowptr, col = ctx.saved_tensors
        dout = dout.contiguous()
        N, F = x.shape
        H, C = al.shape[-2], al.shape[-1]
        D = H * C
        dev = x.device
        s = _lib.stream(dev)
        delta = torch.empty((N, H), dtype=torch.float32, device=dev)
        da_dst = torch.empty_like(delta)
        with _timed("gat_agg_bwd_dst"):
            _lib.check(lib.hicgat_gat_agg_bwd_dst(_lib.ptr(rowptr), _lib.ptr(col), N, H, C, _lib.ptr(h),
                                                  _lib.ptr(a_src), _lib.ptr(a_dst), _lib.ptr(rmax),
                                                  _lib.ptr(rsum), _lib.ptr(dout), ctx.ns, _lib.ptr(delta),
                                                  _lib.ptr(da_dst), s), "hicgat_gat_agg_bwd_dst")
        dh = torch.empty((N, D), dtype=torch.float32, device=dev)
        da_src = torch.empty_like(delta)
        with _timed("gat_agg_bwd_src"):
            _lib.check(lib.hicgat_gat_agg_bwd_src(_lib.ptr(rowptr), _lib.ptr(col), N, H, C, _lib.ptr(h),
                                                  _lib.ptr(a_src), _lib.ptr(a_dst), _lib.ptr(rmax),
                                                  _lib.ptr(rsum), _lib.ptr(delta), _lib.ptr(da_dst),
                                                  _lib.ptr(dout), _lib.ptr(al), _lib.ptr(ar), ctx.ns,
                                                  _lib.ptr(dh), _lib.ptr(da_src), s), "hicgat_gat_agg_bwd_src")
        datt_l = torch.empty((D,), dtype=torch.float32, device=dev)
        datt_r = torch.empty_like(datt_l)
        dbias = torch.empty_like(datt_l)
        ws = _lib.workspace(lib.hicgat_gat_param_grad_workspace_bytes(N, D), dev)
        _lib.check(lib.hicgat_gat_param_grad(_lib.ptr(h), _lib.ptr(dout), _lib.ptr(da_src), _lib.ptr(da_dst),
                                             N, H, C, _lib.ptr(datt_l), _lib.ptr(datt_r), _lib.ptr(dbias),
                                             _lib.ptr(ws), ws.numel(), s), "hicgat_gat_param_grad")
        dW = dh.t().mm(x) if ctx.needs_input_grad[1] else None
        dx = dh.mm(W) if ctx.needs_input_grad[0] else None
        return (dx, dW, datt_l.view(al.shape), datt_r.view(ar.shape),
                dbias if ctx.has_bias else None, None, None, None)


def gat_conv(x, W, att_l, att_r, bias, adj, negative_slope=0.2):
    if adj.rowptr32 is None or adj.rowptr32.device != x.device:
        adj.to(x.device)
    return _GATConvFn.apply(x, W, att_l, att_r, bias, adj.rowptr32, adj.col32, negative_slope)


class _PairDistFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords):
        lib = _lib.lib()
        _dev_check(coords)
        c = coords.contiguous().float()
        n = c.shape[0]
        D = torch.empty((n, n), dtype=torch.float32, device=c.device)
        _lib.check(lib.hicgat_pairdist_fwd(_lib.ptr(c), n, _lib.ptr(D), n, _lib.stream(c.device)),
                   "hicgat_pairdist_fwd")
        ctx.save_for_backward(c)
        return D

    @staticmethod
    def backward(ctx, dD):
        lib = _lib.lib()
        (c,) = ctx.saved_tensors
        n = c.shape[0]
        g = dD.contiguous().float()
        dc = torch.empty_like(c)
        ws = _lib.workspace(lib.hicgat_pairdist_workspace_bytes(n, 0), c.device)
        _lib.check(lib.hicgat_pairdist_bwd(_lib.ptr(c), _lib.ptr(g), n, n, _lib.ptr(dc), _lib.ptr(ws),
                                           ws.numel(), _lib.stream(c.device)), "hicgat_pairdist_bwd")
        return dc


def pairwise_dist(coords):
    """torch.cdist(coords, coords, p=2) on the GPU (models.py:661)."""
    return _PairDistFn.apply(coords)


class _FusedLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords, tbuf, n, loss_kind, tile_begin, tile_end, stats):
        lib = _lib.lib()
        c = coords.contiguous().float()
        dc = torch.empty_like(c)
        loss = torch.empty((), dtype=torch.float32, device=c.device)
        ws = _lib.workspace(lib.hicgat_pairdist_workspace_bytes(n, 1), c.device)
        with _timed("pairdist_mse_fused"):
            _lib.check(lib.hicgat_pairdist_mse_fused(_lib.ptr(c), _lib.ptr(tbuf), n, tbuf.shape[1], tile_begin,
                                                     tile_end, loss_kind, _lib.ptr(stats), _lib.ptr(loss),
                                                     _lib.ptr(dc), _lib.ptr(ws), ws.numel(),
                                                     _lib.stream(c.device)), "hicgat_pairdist_mse_fused")
        ctx.save_for_backward(dc)
        return loss

    @staticmethod
    def backward(ctx, gl):
        (dc,) = ctx.saved_tensors
        return dc * gl, None, None, None, None, None, None


def fused_dist_loss(coords, truth, kind="mse", tile_range=(0, -1), stats=None):
    """MSE(cdist(coords), truth) [kind="mse", HiC-GNN_main.py:127] or
    MSE + alpha*(1 - pearson) [kind="combined", HiC_GAT_generalize_directly.py:219-225] with the
    gradient of the MSE only (the Pearson term is a detached host value in the reference).

    ``truth`` is a ``graph.Truth`` (symmetric).  ``stats`` (float64 [10], device) receives the
    moments, mse, r, alpha and total (see include/hicgat.h)."""
    if not truth.symmetric:
        raise NotImplementedError("fused loss needs a symmetric truth matrix; use pairwise_dist + MSELoss")
    if stats is None:
        stats = torch.empty(10, dtype=torch.float64, device=coords.device)
    kind_i = {"mse": 0, "combined": 1}[kind]
    loss = _FusedLossFn.apply(coords, truth.buf, truth.n, kind_i, int(tile_range[0]), int(tile_range[1]), stats)
    return loss, stats
