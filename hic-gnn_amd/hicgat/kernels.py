"""Row-level launchers of the libhicgat.so kernels (one method per C-ABI entry point family).

``HipKernels`` is what the product runs.  Every method takes and returns device tensors and is
stream-ordered on torch's current stream; the ``timed`` names feed bench.py's live roofline.
The distributed trainer (``hicgat.dist``) is written against this interface only, so its
partitioning / collective logic can be exercised on CPU in tests with a stand-in object.
"""
import os

import torch

from . import _lib

# name -> list of (start, end) torch.cuda.Event pairs recorded around launches (bench.py)
TIMERS = None
GEMM_F32 = 1   # include/hicgat.h HICGAT_GEMM_F32: fp32 MFMA (the only GEMM arithmetic)


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


P = _lib.ptr

# K-split of a node-row GEMM (Linear forward / input gradient: M = rows) that would leave the chip
# mostly idle: a rank's shard of the multi-GPU step (M ~ 2700 rows at P = 8) gives the 64 x 128
# kernel 43 x 4 = 172 workgroups with the whole K = 512 each, one per CU, latency-bound per K-step
# (38 us for 1.4 GFLOP, profiles/r03f_simprof_*_P8_rank0_timeline.txt; split in 3: 28 + 7 us for the slab
# sum).  Split over K until ~512 workgroups are in flight (each split >= 128 deep), partial slabs
# added in split order (deterministic).  The tall 160 x 128 kernel split the same way (a grid.y of
# K-chunks into slabs) measured slower at these shapes (r03i: 23-33 + 8 us) and was not kept.
# Shapes that fill the chip on their own -- every single-GPU shape at N = 20000 (the tall kernel,
# or >= 256 tiles) -- keep splits = 1.  HICGAT_ROW_SPLIT=0: off (A/B).
ROW_SPLIT = os.environ.get("HICGAT_ROW_SPLIT", "1") != "0"
_TALL_MIN_TILES = 192   # gemm.hip tall_min_tiles(): the tall kernel takes shapes with at least this many tiles


def row_splits(M, N, K):
    if not ROW_SPLIT or M < 1024 or K < 256:
        return 1
    if -(-M // 160) * (N // 128) >= _TALL_MIN_TILES:      # the tall kernel takes it (gemm.hip dispatch)
        return 1
    wgs = -(-M // 64) * -(-N // (128 if N >= 128 else 64))
    if wgs >= 256:
        return 1
    return max(1, min(K // 128, -(-512 // wgs)))


class HipKernels:
    """The MI355X implementation of the kernel interface."""

    def __init__(self):
        self.lib = _lib.lib()
        self.gemm_impl = GEMM_F32

    # -- a2 ---------------------------------------------------------------------------------------
    def linear_att(self, x, W, att_l, att_r, h=None):
        """h = x W^T (into ``h``, e.g. a rank's rows of the all-gather buffer, if given) + logits."""
        N, F = x.shape
        H, C = att_l.shape[-2], att_l.shape[-1]
        if h is None:
            h = torch.empty((N, H * C), dtype=torch.float32, device=x.device)
        assert h.shape == (N, H * C) and h.is_contiguous()
        a_src = torch.empty((N, H), dtype=torch.float32, device=x.device)
        a_dst = torch.empty_like(a_src)
        if N >= 32 and F % 4 == 0 and x.stride(0) % 4 == 0:
            # the tall 160x128 GEMM into h, then the logits in one pass over h (2.075 vs 2.095 ms per
            # step for the 64x256-tile hicgat_gat_linear_att with the logits in its epilogue, which
            # takes the small / unaligned cases)
            st = _lib.stream(x.device)
            with _timed("gat_linear_att"):
                _lib.check(self.lib.hicgat_gemm_ex(0, 0, N, H * C, F, P(x), x.stride(0), P(W), W.stride(0), None, P(h),
                                                   h.stride(0), 0, 1, self.gemm_impl, None, 0, st), "hicgat_gemm_ex")
                _lib.check(self.lib.hicgat_gat_att_logits(P(h), P(att_l), P(att_r), N, H, C, P(a_src), P(a_dst), st),
                           "hicgat_gat_att_logits")
            return h, a_src, a_dst
        with _timed("gat_linear_att"):
            _lib.check(self.lib.hicgat_gat_linear_att(P(x), P(W), P(att_l), P(att_r), N, F, H, C, P(h), P(a_src),
                                                      P(a_dst), _lib.stream(x.device)), "hicgat_gat_linear_att")
        return h, a_src, a_dst

    def att_logits(self, h, att_l, att_r):
        N = h.shape[0]
        H, C = att_l.shape[-2], att_l.shape[-1]
        a_src = torch.empty((N, H), dtype=torch.float32, device=h.device)
        a_dst = torch.empty_like(a_src)
        _lib.check(self.lib.hicgat_gat_att_logits(P(h), P(att_l), P(att_r), N, H, C, P(a_src), P(a_dst),
                                                  _lib.stream(h.device)), "hicgat_gat_att_logits")
        return a_src, a_dst

    # -- a4 + a5 ----------------------------------------------------------------------------------
    def agg_fwd(self, rowptr, col, r0, r1, h, a_src, a_dst, bias, ns, out, row_stats):
        N = h.shape[0]
        H = a_src.shape[1]
        C = h.shape[1] // H
        with _timed("gat_agg_fwd"):
            _lib.check(self.lib.hicgat_gat_agg_fwd(P(rowptr), P(col), N, col.numel(), H, C, r0, r1, P(h), P(a_src),
                                                   P(a_dst), P(bias), float(ns), P(out), P(row_stats),
                                                   _lib.stream(h.device)), "hicgat_gat_agg_fwd")

    def agg_fwd_act(self, rowptr, col, r0, r1, h, a_src, a_dst, bias, ns, act, out, out2, row_stats):
        """Training form: ``act`` 1 = relu epilogue; ``out2`` (or None) = sum alpha lrelu' h."""
        N = h.shape[0]
        H = a_src.shape[1]
        C = h.shape[1] // H
        with _timed("gat_agg_fwd"):
            _lib.check(self.lib.hicgat_gat_agg_fwd_act(P(rowptr), P(col), N, col.numel(), H, C, r0, r1, P(h),
                                                       P(a_src), P(a_dst), P(bias), float(ns), int(act), P(out),
                                                       P(out2), P(row_stats), _lib.stream(h.device)),
                       "hicgat_gat_agg_fwd_act")

    def agg_fwd_tiled(self, rowptr, col, tiles, h, a_src, a_dst, bias, ns, act, out, out2, row_stats):
        """``agg_fwd_act`` over rows [tiles.r0, tiles.r1) with the dense tiles on the matrix cores."""
        N = h.shape[0]
        H = a_src.shape[1]
        C = h.shape[1] // H
        t = tiles
        ws = self.tiled_workspace(t, h.device)
        with _timed("gat_agg_fwd"):
            _lib.check(self.lib.hicgat_gat_agg_fwd_tiled(
                P(rowptr), P(col), P(t.rowptr_s), P(t.col_s), P(t.tptr), P(t.tcol), P(t.tmask), t.ntiles, N, H, C,
                t.r0, t.r1, P(h), P(a_src), P(a_dst), P(bias), float(ns), int(act), P(out), P(out2), P(row_stats),
                t.splits, P(ws), 0 if ws is None else ws.numel(), _lib.stream(h.device)), "hicgat_gat_agg_fwd_tiled")

    def tiled_workspace(self, t, device):
        nb = self.lib.hicgat_gat_tiled_workspace_bytes(t.r1 - t.r0, t.splits)
        return _lib.workspace(nb, device) if nb else None

    def agg_bwd_src_tiled(self, tiles, h, a_src, a_dst, row_stats, dout, att_l, att_r, ns, dh, da_src):
        """``agg_bwd_src`` over rows [tiles.r0, tiles.r1) with the dense tiles on the matrix cores."""
        N = h.shape[0]
        H = a_src.shape[1]
        C = h.shape[1] // H
        assert row_stats.stride(1) == 1 and dout.stride(1) == 1
        t = tiles
        ws = self.tiled_workspace(t, h.device)
        with _timed("gat_agg_bwd_src"):
            _lib.check(self.lib.hicgat_gat_agg_bwd_src_tiled(
                P(t.rowptr_s), P(t.col_s), P(t.tptr), P(t.tcol), P(t.tmask), t.ntiles, N, H, C, t.r0, t.r1, P(h),
                P(a_src), P(a_dst), P(row_stats), row_stats.stride(0), P(dout), dout.stride(0), P(att_l), P(att_r),
                float(ns), P(dh), P(da_src), t.splits, P(ws), 0 if ws is None else ws.numel(),
                _lib.stream(h.device)), "hicgat_gat_agg_bwd_src_tiled")

    def agg_bwd_rows(self, r0, r1, act, g, y, bias, out2, dout, row_stats):
        """Destination half of the backward without a gather (after ``agg_fwd_act`` with out2);
        ``dout`` (act = 1) may be a row-strided view, e.g. the dout columns of a packed buffer."""
        N, D = y.shape
        H = row_stats.shape[1] // 4
        assert row_stats.stride(0) == 4 * H and y.stride(0) == D
        with _timed("gat_agg_bwd_rows"):
            _lib.check(self.lib.hicgat_gat_agg_bwd_rows(N, H, D // H, r0, r1, int(act), P(g), P(y), P(bias), P(out2),
                                                        P(dout), 0 if dout is None else dout.stride(0),
                                                        P(row_stats), _lib.stream(y.device)),
                       "hicgat_gat_agg_bwd_rows")

    def agg_bwd_dst(self, rowptr, col, r0, r1, h, a_src, a_dst, dout, ns, row_stats):
        N = h.shape[0]
        H = a_src.shape[1]
        C = h.shape[1] // H
        with _timed("gat_agg_bwd_dst"):
            _lib.check(self.lib.hicgat_gat_agg_bwd_dst(P(rowptr), P(col), N, H, C, r0, r1, P(h), P(a_src),
                                                       P(a_dst), P(dout), float(ns), P(row_stats),
                                                       _lib.stream(h.device)), "hicgat_gat_agg_bwd_dst")

    SRC_ROUND_ROBIN = 1   # include/hicgat.h HICGAT_SRC_ROUND_ROBIN

    def agg_bwd_src(self, rowptr, col, r0, r1, h, a_src, a_dst, row_stats, dout, att_l, att_r, ns, dh, da_src,
                    round_robin=False):
        """``round_robin``: row blocks spread over the XCDs (the multi-GPU slab pass, hicgat.dist)."""
        N = h.shape[0]
        H = a_src.shape[1]
        C = h.shape[1] // H
        # row_stats / dout may be row-strided views (the packed all-gather buffer of hicgat.dist)
        assert row_stats.stride(1) == 1 and dout.stride(1) == 1
        with _timed("gat_agg_bwd_src"):
            _lib.check(self.lib.hicgat_gat_agg_bwd_src_ex(P(rowptr), P(col), N, H, C, r0, r1, P(h), P(a_src),
                                                          P(a_dst), P(row_stats), row_stats.stride(0), P(dout),
                                                          dout.stride(0), P(att_l), P(att_r), float(ns), P(dh),
                                                          P(da_src), self.SRC_ROUND_ROBIN if round_robin else 0,
                                                          _lib.stream(h.device)),
                       "hicgat_gat_agg_bwd_src_ex")

    def param_grad(self, h, dout, da_src, row_stats, H, out=None, accumulate=False):
        """Column sums over the given rows -> (datt_src [D], datt_dst [D], dbias [D]); ``out`` =
        three destination tensors (e.g. the parameters' own .grad views) to write or add into; a
        None among them skips that part (datt_dst / dbias need no source-pass output)."""
        N, D = h.shape
        C = D // H
        dev = h.device
        if out is None:
            out = tuple(torch.empty(D, dtype=torch.float32, device=dev) for _ in range(3))
        datt_l, datt_r, dbias = out
        ws = _lib.workspace(self.lib.hicgat_gat_param_grad_workspace_bytes(N, D), dev)
        with _timed("param_grad"):
            _lib.check(self.lib.hicgat_gat_param_grad(P(h), P(dout), P(da_src), P(row_stats), N, H, C, P(datt_l),
                                                      P(datt_r), P(dbias), int(accumulate), P(ws), ws.numel(),
                                                      _lib.stream(dev)), "hicgat_gat_param_grad")
        return datt_l, datt_r, dbias

    # -- aggregate-first GATConv (gat_xagg.hip): the multi-GPU "xagg" step (hicgat.dist) ---------------
    def xagg_logits(self, x, W, att_l, att_r, a_src, a_dst, zero=None, step_ctr=None, pack=None):
        """a_src / a_dst [N, 2] = x . (W_h^T att^h) for every row of x; ``zero``: a contiguous buffer
        zeroed in the same launch (the step's flat gradient buffer); ``step_ctr``: the optimizer's
        device step count, advanced in the same launch (its Adam then runs with ``counted=True``);
        ``pack`` ((W1c, W2c, _, buffer), ``ops.step_pack``): the head-fused tail's packed weights of
        W1c, W2c and W written into the buffer by the same launch."""
        N, F = x.shape
        H, C = att_l.shape[-2], att_l.shape[-1]
        vec = _lib.workspace(self.lib.hicgat_xagg_vec_bytes(), x.device)
        assert zero is None or zero.is_contiguous()
        W1c = W2c = buf = None
        nb = 0
        if pack is not None:
            W1c, W2c, _, buf = pack
            assert W.is_contiguous() and W1c.is_contiguous() and W2c.is_contiguous()
            nb = buf.numel() * buf.element_size()
        with _timed("xagg_logits"):
            _lib.check(self.lib.hicgat_xagg_logits_zero_pack(
                P(x), P(W), P(att_l), P(att_r), N, F, H, C, P(vec), P(a_src), P(a_dst), P(zero),
                0 if zero is None else zero.numel(), P(step_ctr), P(W1c), P(W2c), P(buf), nb,
                _lib.stream(x.device)), "hicgat_xagg_logits_zero_pack")

    def xagg_fwd(self, rowptr, col, r0, r1, x, a_src, a_dst, ns, X4, row_stats):
        """Own rows [r0, r1): X4 [2, 2, r1 - r0, 512] = (xa, xa2) per head; row stats (global rows)."""
        N, F = x.shape
        assert X4.shape == (2, 2, r1 - r0, F) and X4.is_contiguous() and row_stats.shape[0] == N
        with _timed("gat_agg_fwd"):
            _lib.check(self.lib.hicgat_xagg_fwd(P(rowptr), P(col), N, F, 2, F // 2, r0, r1, P(x), P(a_src), P(a_dst),
                                                float(ns), P(X4), P(row_stats), _lib.stream(x.device)),
                       "hicgat_xagg_fwd")

    def xagg_bias_relu(self, y0, bias, o):
        rows, D = y0.shape
        assert y0.is_contiguous() and o.is_contiguous() and o.shape == y0.shape
        _lib.check(self.lib.hicgat_xagg_bias_relu(P(y0), P(bias), P(o), rows, D, _lib.stream(y0.device)),
                   "hicgat_xagg_bias_relu")

    def xagg_rows_bwd(self, act, g, y0, bias, dout, row_stats):
        """Own rows: dout = g relu'(y0) (act) or g, delta -> row_stats[:, 4:6], S3 -> [:, 6:8]."""
        rows, D = y0.shape
        assert row_stats.shape == (rows, 8) and row_stats.is_contiguous()
        with _timed("gat_agg_bwd_rows"):
            _lib.check(self.lib.hicgat_xagg_rows_bwd(rows, D, int(act), P(g), P(y0), P(bias), P(dout), P(row_stats),
                                                     _lib.stream(y0.device)), "hicgat_xagg_rows_bwd")

    def xagg_edge(self, rowptr, col, r0, r1, x, a_src, a_dst, row_stats, dxa, ns, ds, xa2=None):
        """Per-edge softmax terms of own rows; with ``xa2`` (X4[:, 1]) also da_dst (row_stats[:, 6:8])."""
        N, F = x.shape
        assert dxa.shape == (r1 - r0, 2 * F) and dxa.is_contiguous()
        with _timed("gat_agg_bwd_dst"):
            _lib.check(self.lib.hicgat_xagg_edge(P(rowptr), P(col), N, F, 2, F // 2, r0, r1, P(x), P(a_src), P(a_dst),
                                                 P(row_stats), P(dxa), P(xa2), float(ns), P(ds), _lib.stream(x.device)),
                       "hicgat_xagg_edge")

    def xagg_edge_acc(self, rowptr, col, r0, r1, x, a_src, a_dst, row_stats, dxa, ns, gpart, xa2=None):
        """The edge pass with g_src's partial rows (``gpart`` [edge_acc_blocks, 1024]); with ``xa2``
        also da_dst (row_stats[:, 6:8])."""
        N, F = x.shape
        assert dxa.shape == (r1 - r0, 2 * F) and dxa.is_contiguous()
        assert gpart.shape == (self.edge_acc_blocks(r1 - r0), 2 * F) and gpart.is_contiguous()
        with _timed("gat_agg_bwd_dst"):
            _lib.check(self.lib.hicgat_xagg_edge_acc(P(rowptr), P(col), N, F, 2, F // 2, r0, r1, P(x), P(a_src),
                                                     P(a_dst), P(row_stats), P(dxa), P(xa2), float(ns), P(gpart),
                                                     _lib.stream(x.device)), "hicgat_xagg_edge_acc")

    def edge_acc_blocks(self, rows):
        """Partial rows of g_src that hicgat_xagg_edge_acc writes for ``rows`` own rows."""
        return int(self.lib.hicgat_xagg_edge_acc_blocks(int(rows)))

    def xagg_slab_sum(self, rowptr_s, perm, ds, x, da_src, g_src):
        """da_src (every row, through the slab) and g_src [2, 512] = sum_j da_src_j x_j."""
        N = da_src.shape[0]
        ws = _lib.workspace(self.lib.hicgat_xagg_slab_workspace_bytes(), ds.device)
        with _timed("gat_agg_bwd_src"):
            _lib.check(self.lib.hicgat_xagg_slab_sum(P(rowptr_s), P(perm), N, P(ds), P(x), P(da_src), P(g_src), P(ws),
                                                     ws.numel(), _lib.stream(ds.device)), "hicgat_xagg_slab_sum")

    def xagg_param_finish(self, W, att_l, att_r, g_src, g_dst, dW, datt_l, datt_r):
        """``g_src`` / ``g_dst``: [2 * 512] or, segmented, [segs, 2 * 512] views (the segments are added)."""
        H, C = att_l.shape[-2], att_l.shape[-1]
        if g_src.dim() == 2:
            assert g_dst.shape == g_src.shape and g_src.stride(0) == g_dst.stride(0) and g_src.stride(1) == 1
            _lib.check(self.lib.hicgat_xagg_param_finish_seg(P(W), P(att_l), P(att_r), P(g_src), P(g_dst),
                                                             g_src.shape[0], g_src.stride(0), W.shape[1], H, C, P(dW),
                                                             P(datt_l), P(datt_r), _lib.stream(W.device)),
                       "hicgat_xagg_param_finish_seg")
            return
        _lib.check(self.lib.hicgat_xagg_param_finish(P(W), P(att_l), P(att_r), P(g_src), P(g_dst), W.shape[1], H, C,
                                                     P(dW), P(datt_l), P(datt_r), _lib.stream(W.device)),
                   "hicgat_xagg_param_finish")

    # -- f1: SAGEConv (layers.py:41-79) --------------------------------------------------------------
    def sage_weights(self, A, rowptr, col):
        n = A.shape[0]
        w = torch.empty(col.numel(), dtype=torch.float32, device=A.device)
        inv = torch.empty(n, dtype=torch.float32, device=A.device)
        _lib.check(self.lib.hicgat_sage_weights(P(A), n, A.stride(0), P(rowptr), P(col), P(w), P(inv),
                                                _lib.stream(A.device)), "hicgat_sage_weights")
        return w, inv

    def sage_agg(self, rowptr, col, w, inv, r0, r1, x, z, transpose=False, write_trunc=False):
        N, F = x.shape
        with _timed("sage_agg"):
            _lib.check(self.lib.hicgat_sage_agg(P(rowptr), P(col), P(w), P(inv), N, F, r0, r1, P(x), int(transpose),
                                                int(write_trunc), P(z), z.stride(0), _lib.stream(x.device)),
                       "hicgat_sage_agg")
        return z

    # -- a7..a9 -----------------------------------------------------------------------------------
    PD_SQUARE, PD_TRI = 0, 1   # include/hicgat.h HICGAT_PD_*

    def num_tiles(self, n):
        """Upper-triangle 128 x 128 tiles of the fused loss (a rank takes a contiguous range)."""
        return int(self.lib.hicgat_pairdist_num_tiles(n, self.PD_TRI))

    def fused_loss(self, coords, tbuf, n, kind, t0, t1, stats, loss, dcoords, row0=0, col0=0):
        """``tbuf`` is the truth or a band of it starting at (row0, col0) (hicgat.dist)."""
        ws = _lib.workspace(self.lib.hicgat_pairdist_workspace_bytes(n, self.PD_TRI), coords.device)
        with _timed("pairdist_mse_fused"):
            _lib.check(self.lib.hicgat_pairdist_mse_fused_band(
                P(coords), P(tbuf), n, tbuf.shape[1], int(row0), tbuf.shape[0], int(col0), int(t0), int(t1),
                int(kind), P(stats), P(loss), P(dcoords), P(ws), ws.numel(), _lib.stream(coords.device)),
                "hicgat_pairdist_mse_fused_band")

    def fused_loss_support(self, coords, sf, n, kind, stats, loss, dcoords):
        """The fused loss over a truth in background + support form (``graph.SupportForm``)."""
        ws = _lib.workspace(self.lib.hicgat_pairdist_support_workspace_bytes(n), coords.device)
        with _timed("pairdist_mse_fused"):
            _lib.check(self.lib.hicgat_pairdist_mse_fused_support_range_ex(
                P(coords), None, n, sf.background, P(sf.rowptr), P(sf.col_buf), P(sf.val_buf), P(sf.diag), 0, -1, 0,
                n, int(kind), P(stats), P(loss), P(dcoords), None, P(ws), ws.numel(),
                _lib.stream(coords.device)), "hicgat_pairdist_mse_fused_support_range_ex")

    def fused_loss_support_range(self, coords, sf, n, kind, t0, t1, s0, s1, stats, loss, dcoords, cmap=None):
        """A rank's share of the background-form loss: bulk tiles [t0, t1), support rows [s0, s1)
        (partial moments and dcoords; the caller all-reduces them and calls ``loss_finalize``).
        A float64 ``dcoords`` receives the fp32 gradient values widened (one all-reduce buffer);
        ``cmap`` (int32 [n]): global row -> row of ``coords``."""
        ws = _lib.workspace(self.lib.hicgat_pairdist_support_workspace_bytes(n), coords.device)
        d32, d64 = (None, dcoords) if dcoords.dtype == torch.float64 else (dcoords, None)
        assert cmap is None or (cmap.dtype == torch.int32 and cmap.numel() == n)
        with _timed("pairdist_mse_fused"):
            _lib.check(self.lib.hicgat_pairdist_mse_fused_support_range_ex(
                P(coords), P(cmap), n, sf.background, P(sf.rowptr), P(sf.col_buf), P(sf.val_buf), P(sf.diag), int(t0),
                int(t1), int(s0), int(s1), int(kind), P(stats), P(loss), P(d32), P(d64), P(ws), ws.numel(),
                _lib.stream(coords.device)), "hicgat_pairdist_mse_fused_support_range_ex")

    def loss_finalize(self, n, kind, stats, loss, dc64=None, r0=0, r1=0, dcoords=None, reorder=None):
        """mse / r / alpha / total from the (all-reduced) moments; with ``dc64`` also dcoords[r0:r1] =
        fp32(dc64[r0:r1]) in the same launch; ``reorder`` = (cbuf, gidx32, cglob): also cglob[i] =
        cbuf[gidx[i]] (the all-gathered coordinates in global row order)."""
        if dc64 is None:
            _lib.check(self.lib.hicgat_pairdist_finalize(n, int(kind), P(stats), P(loss), _lib.stream(stats.device)),
                       "hicgat_pairdist_finalize")
            return
        assert dc64.is_contiguous() and dcoords.is_contiguous() and dc64.shape == dcoords.shape == (n, 3)
        cbuf, gidx, cglob = reorder if reorder is not None else (None, None, None)
        if reorder is not None:
            assert cbuf.is_contiguous() and cglob.shape == (n, 3) and gidx.dtype == torch.int32 and gidx.numel() == n
        _lib.check(self.lib.hicgat_pairdist_finalize_rows_ex(n, int(kind), P(stats), P(loss), P(dc64), int(r0), int(r1),
                                                             P(dcoords), P(cbuf), P(gidx), P(cglob),
                                                             _lib.stream(stats.device)),
                   "hicgat_pairdist_finalize_rows_ex")

    def pairdist_fwd(self, coords):
        n = coords.shape[0]
        D = torch.empty((n, n), dtype=torch.float32, device=coords.device)
        _lib.check(self.lib.hicgat_pairdist_fwd(P(coords), n, P(D), n, _lib.stream(coords.device)),
                   "hicgat_pairdist_fwd")
        return D

    def pairdist_bwd(self, coords, G):
        n = coords.shape[0]
        dc = torch.empty_like(coords)
        ws = _lib.workspace(self.lib.hicgat_pairdist_workspace_bytes(n, self.PD_SQUARE), coords.device)
        _lib.check(self.lib.hicgat_pairdist_bwd(P(coords), P(G), n, G.shape[1], P(dc), P(ws), ws.numel(),
                                                _lib.stream(coords.device)), "hicgat_pairdist_bwd")
        return dc

    # -- a6: Linear layers on the MFMA GEMM (fp32, or the fp32-accurate x3 split) ------------------
    def gemm(self, a_kmajor, b_kmajor, M, N, K, A, B, C, bias=None, accumulate=False, splits=None, name="gemm",
             impl=None):
        """``splits=None``: ``row_splits`` for node-row (row-major A) fp32 problems, else 1; an int is
        taken as given."""
        dev = C.device
        ws = None
        impl = self.gemm_impl if impl is None else impl
        if splits is None:
            splits = row_splits(M, N, K) if (not a_kmajor and impl == 1) else 1
        if splits > 1:
            ws = _lib.workspace(self.lib.hicgat_gemm_workspace_bytes(M, N, splits), dev)
        with _timed(name):
            _lib.check(self.lib.hicgat_gemm_ex(int(a_kmajor), int(b_kmajor), M, N, K, P(A), A.stride(0), P(B),
                                               B.stride(0), P(bias), P(C), C.stride(0), int(accumulate), int(splits),
                                               int(impl), P(ws), 0 if ws is None else ws.numel(), _lib.stream(dev)),
                       "hicgat_gemm_ex")
        return C

    def wgrad(self, dy, x, W_out, b_out=None, accumulate=False, splits=1):
        """dW = dy^T x and db = column sums of dy (``b_out`` may be None) in one split-K GEMM."""
        K_, M = dy.shape
        N = x.shape[1]
        dev = W_out.device
        ws = None
        if splits > 1:
            ws = _lib.workspace(self.lib.hicgat_gemm_wgrad_workspace_bytes(M, N, splits), dev)
        with _timed("gemm_dw"):
            _lib.check(self.lib.hicgat_gemm_wgrad(M, N, K_, P(dy), dy.stride(0), P(x), x.stride(0), P(W_out),
                                                  W_out.stride(0), P(b_out), int(accumulate), int(splits), P(ws),
                                                  0 if ws is None else ws.numel(), _lib.stream(dev)),
                       "hicgat_gemm_wgrad")
        return W_out, b_out

    # workgroups of the grouped weight-gradient launch (hicgat_param_grads_grouped): ~2 per CU
    GROUP_WGS = int(os.environ.get("HICGAT_GROUP_WGS", "512"))
    # target workgroups of a grouped node-row GEMM launch (sets its K split; 0 = no split: the tiles
    # write C, bias and relu copy themselves and the slab-sum launch goes away)
    ROWS_WGS = int(os.environ.get("HICGAT_ROWS_WGS", "512"))
    SMALL_M = 16

    def param_grads_grouped(self, wjobs, cjobs, target_wgs=None, small_m=None):
        """Every queued parameter gradient of a step in two launches (include/hicgat.h
        hicgat_param_grads_grouped): ``wjobs`` = [(dy [K, M], x [K, N], dW [M, N], db [M] or None,
        accumulate)], ``cjobs`` = [(src [rows, cols], dst [cols], accumulate[, wt [rows] view])].
        A weight gradient of fewer than ``SMALL_M`` output rows (dense3: 3, g_dst: 2) becomes M
        weighted column sums (and a plain one for db) instead of a 128 x 128 MFMA tile that would
        be 97 % padding (``small_m``: that bound, default ``SMALL_M``; 0: every job a tile -- the
        tall weighted sums of a 20 000-row step are long single-block chains)."""
        target = self.GROUP_WGS if target_wgs is None else target_wgs
        small_m = self.SMALL_M if small_m is None else small_m
        big, cjobs = [], list(cjobs)
        for dy, x, dw, db, acc in wjobs:
            if dy.shape[1] < small_m:
                cjobs += [(x, dw[m], acc, dy[:, m]) for m in range(dy.shape[1])]
                if db is not None:
                    cjobs.append((dy, db, acc))
            else:
                big.append((dy, x, dw, db, acc))
        wjobs = big
        W = (_lib.WgradJob * max(1, len(wjobs)))()
        for k, (dy, x, dw, db, acc) in enumerate(wjobs):
            assert dy.stride(1) == 1 and x.stride(1) == 1 and dw.stride(1) == 1 and dy.shape[0] == x.shape[0]
            assert db is None or db.is_contiguous()
            W[k] = _lib.WgradJob(dy.data_ptr(), dy.stride(0), x.data_ptr(), x.stride(0), dw.data_ptr(), dw.stride(0),
                                 None if db is None else db.data_ptr(), dy.shape[1], x.shape[1], dy.shape[0], int(acc))
        C = (_lib.ColsumJob * max(1, len(cjobs)))()
        for k, job in enumerate(cjobs):
            src, dst, acc = job[:3]
            wt = job[3] if len(job) > 3 else None
            assert src.dim() == 2 and src.stride(1) == 1
            if dst.dim() == 2:    # [segs, cols]: the rows summed in segs segments, one dst row each
                assert dst.stride(1) == 1 and dst.shape[1] == src.shape[1] and 1 <= dst.shape[0] <= max(1, src.shape[0])
                segs, ldd = dst.shape[0], dst.stride(0)
            else:
                assert dst.is_contiguous() and dst.numel() == src.shape[1]
                segs, ldd = 1, 0
            assert wt is None or (wt.dim() == 1 and wt.shape[0] == src.shape[0])
            C[k] = _lib.ColsumJob(src.data_ptr(), src.stride(0), src.shape[0], src.shape[1], dst.data_ptr(), int(acc),
                                  None if wt is None else wt.data_ptr(), 0 if wt is None else wt.stride(0), segs, ldd)
        dev = (wjobs[0][0] if wjobs else cjobs[0][0]).device
        ws = _lib.workspace(self.lib.hicgat_param_grads_workspace_bytes(W, len(wjobs), target), dev)
        with _timed("param_grads_grouped"):
            _lib.check(self.lib.hicgat_param_grads_grouped(W, len(wjobs), C, len(cjobs), int(target), P(ws), ws.numel(),
                                                           _lib.stream(dev)), "hicgat_param_grads_grouped")

    def gemm_rows_grouped(self, jobs, b_kmajor, splits=None, name="gemm_grouped"):
        """include/hicgat.h hicgat_gemm_rows_grouped: ``jobs`` = [(A [M, K], B, C [M, N], bias or None,
        C_relu or None)], B [N, K] (``b_kmajor`` 0) or [K, N] (1).  ``splits`` None: enough K chunks
        for ~512 workgroups over all jobs (each chunk >= 128 deep)."""
        G = (_lib.GemmJob * len(jobs))()
        wgs = 0
        for k, (A, B, C, bias, Cr) in enumerate(jobs):
            M, Kd = A.shape
            N = C.shape[1]
            assert A.stride(1) == 1 and B.stride(1) == 1 and C.stride(1) == 1 and C.shape[0] == M
            assert (B.shape == (N, Kd)) if not b_kmajor else (B.shape == (Kd, N))
            assert Cr is None or (Cr.shape == C.shape and Cr.stride(1) == 1)
            G[k] = _lib.GemmJob(A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), C.data_ptr(), C.stride(0),
                                None if Cr is None else Cr.data_ptr(), 0 if Cr is None else Cr.stride(0),
                                None if bias is None else bias.data_ptr(), M, N, Kd)
            wgs += -(-M // 64) * -(-N // 128)
        if splits is None:
            splits = max(1, min(jobs[0][0].shape[1] // 128, -(-self.ROWS_WGS // max(1, wgs)))) if self.ROWS_WGS else 1
        dev = jobs[0][2].device
        ws = _lib.workspace(self.lib.hicgat_gemm_rows_grouped_workspace_bytes(G, len(jobs), splits), dev)
        with _timed(name):
            _lib.check(self.lib.hicgat_gemm_rows_grouped(G, len(jobs), int(b_kmajor), int(splits), P(ws), ws.numel(),
                                                         _lib.stream(dev)), "hicgat_gemm_rows_grouped")

    def colsum(self, A, out, accumulate=False):
        K, N = A.shape
        ws = _lib.workspace(self.lib.hicgat_colsum_workspace_bytes(K, N), A.device)
        with _timed("colsum"):
            _lib.check(self.lib.hicgat_colsum(P(A), A.stride(0), K, N, P(out), int(accumulate), P(ws), ws.numel(),
                                              _lib.stream(A.device)), "hicgat_colsum")
        return out

    def ln_relu_res_fwd(self, y, gamma, beta, eps, res, z, row_stats):
        M, W = z.shape
        _lib.check(self.lib.hicgat_ln_relu_res_fwd(P(y), y.stride(0), M, W, P(gamma), P(beta), float(eps), P(res),
                                                   0 if res is None else res.stride(0), P(z), P(row_stats),
                                                   _lib.stream(z.device)), "hicgat_ln_relu_res_fwd")

    def ln_relu_res_bwd(self, dz, y, row_stats, gamma, beta, dy, dgamma, dbeta, accumulate=False, dres=None,
                        ws=None):
        """dgamma = dbeta = None: dy / dres only, the partials stay in ``ws`` (pass it, then
        ``ln_relu_res_bwd_params(W, dgamma, dbeta, ws)`` -- on another stream if wanted)."""
        M, W = dz.shape
        if ws is None:
            ws = self.ln_workspace(W, dz.device)
        _lib.check(self.lib.hicgat_ln_relu_res_bwd(P(dz), P(y), y.stride(0), M, W, P(row_stats), P(gamma), P(beta),
                                                   P(dy), dy.stride(0), P(dres), 0 if dres is None else dres.stride(0),
                                                   P(dgamma), P(dbeta), int(accumulate), P(ws), ws.numel(),
                                                   _lib.stream(dz.device)), "hicgat_ln_relu_res_bwd")

    def tail_pack(self, W1c, W2c, Wh=None):
        """The packed copies of W1c [512, 512], W2c [256, 256] and (head forms) Wh [512, 512] that the
        tail kernels read instead of the row-major weights (hicgat_tail_pack): a new device buffer, so
        a forward's copy stays valid for its own backward."""
        for t in (W1c, W2c) + ((Wh,) if Wh is not None else ()):
            assert t.is_contiguous() and t.dtype == torch.float32
        assert W1c.shape == (512, 512) and W2c.shape == (256, 256) and (Wh is None or Wh.shape == (512, 512))
        n = int(self.lib.hicgat_tail_pack_bytes())
        pack = torch.empty(n // 4, dtype=torch.float32, device=W1c.device)
        _lib.check(self.lib.hicgat_tail_pack(P(W1c), P(W2c), P(Wh), P(pack), n, _lib.stream(W1c.device)),
                   "hicgat_tail_pack")
        return pack

    def tail_fwd_fused(self, x, W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4, eps, coords=None,
                       heads=None, pack=None):
        """The flagship's MLP tail forward in one launch (tail_fused.hip): returns (coords, saved)
        with saved = (Y1, st1, z1, Y2, st2, z2, y3, st3, z3); ``coords`` (contiguous [M, 3]): write
        the output there (e.g. the rank's rows of the sharded step's all-gather buffer).
        ``heads`` (``ops.TailHeads``): the head-fused form -- the input rows x (written) are
        relu(xa^h W_h^T + b^h) of the xagg GATConv (hicgat_tail_fwd_fused_heads).  ``pack``: the
        ``tail_pack`` copies of these W1c / W2c (/ the heads' W), or None (row-major reads)."""
        M = x.shape[0]
        dev = x.device
        f = dict(dtype=torch.float32, device=dev)
        Y1, z1 = torch.empty((M, 512), **f), torch.empty((M, 256), **f)
        Y2, z2 = torch.empty((M, 256), **f), torch.empty((M, 128), **f)
        y3, z3 = torch.empty((M, 64), **f), torch.empty((M, 64), **f)
        st1, st2, st3 = (torch.empty((M, 2), **f) for _ in range(3))
        if coords is None:
            coords = torch.empty((M, 3), **f)
        assert coords.shape == (M, 3) and coords.is_contiguous()
        ws = [W1c, b1c, g1, be1, W2c, b2c, g2, be2, W3, b3, g3, be3, W4, b4]
        assert all(t.is_contiguous() for t in ws) and x.stride(1) == 1
        tail = [float(eps), P(Y1), P(st1), P(z1), P(Y2), P(st2), P(z2), P(y3), P(st3), P(z3), P(coords), P(pack),
                _lib.stream(dev)]
        with _timed("tail_fwd_fused"):
            if heads is None:
                _lib.check(self.lib.hicgat_tail_fwd_fused(P(x), x.stride(0), M, *[P(t) for t in ws], *tail),
                           "hicgat_tail_fwd_fused")
            else:
                h = heads
                assert x.is_contiguous() and x.shape == (M, 512) and h.Y0.shape == (M, 512) and h.Y0.is_contiguous()
                assert h.X4.shape[2] == M and h.X4.is_contiguous() and h.W.is_contiguous() and h.bias.is_contiguous()
                _lib.check(self.lib.hicgat_tail_fwd_fused_heads(
                    P(h.X4), h.X4.stride(2), h.X4.stride(0), P(h.W), P(h.bias), P(h.Y0), P(x), M, *[P(t) for t in ws],
                    *tail), "hicgat_tail_fwd_fused_heads")
        return coords, (Y1, st1, z1, Y2, st2, z2, y3, st3, z3)

    def tail_bwd_fused(self, dcoords, saved, W4, W3, W2c, W1c, g1, be1, g2, be2, g3, be3, heads=None, pack=None,
                       rows=None):
        """The tail's input-gradient chain in one launch (tail_fused.hip): returns (dx, dY1, dY2, dy3,
        (ws1, ws2, ws3)) -- the LayerNorm dgamma/dbeta partials stay in the workspaces
        (``ln_relu_res_bwd_params``).  ``heads``: the head-fused form (dx None; the xagg GATConv's
        dout, delta and dxa written into the ``ops.TailHeads`` buffers instead).  ``rows`` = (act, y,
        out2, bias, row_stats, dout): the single-GPU GATConv's rows pass in the epilogue
        (hicgat_tail_bwd_fused_rows; dx None, dout and row_stats[:, 4:8] written instead)."""
        Y1, st1, z1, Y2, st2, z2, y3, st3, z3 = saved
        M = dcoords.shape[0]
        dev = dcoords.device
        f = dict(dtype=torch.float32, device=dev)
        dY1, dY2, dy3 = (torch.empty((M, w), **f) for w in (512, 256, 64))
        dx = torch.empty((M, 512), **f) if heads is None and rows is None else None
        ws = [_lib.workspace(self.lib.hicgat_tail_bwd_workspace_bytes(M, w), dev) for w in (256, 128, 64)]
        ts = [W4, W3, W2c, W1c, g1, be1, g2, be2, g3, be3]
        assert all(t.is_contiguous() for t in ts) and dcoords.is_contiguous()
        wsa = [P(ws[0]), ws[0].numel(), P(ws[1]), ws[1].numel(), P(ws[2]), ws[2].numel()]
        with _timed("tail_bwd_fused"):
            if rows is not None:
                act, y, out2, bias, rs, dout = rows
                for t, w in ((y, 512), (out2, 512), (dout, 512), (rs, 8)):
                    assert t.shape == (M, w) and t.is_contiguous()
                assert bias.is_contiguous() and bias.numel() == 512
                _lib.check(self.lib.hicgat_tail_bwd_fused_rows(
                    P(dcoords), M, P(Y1), P(st1), P(Y2), P(st2), P(y3), P(st3), *[P(t) for t in ts], P(dY1), P(dY2),
                    P(dy3), *wsa, int(act), P(y), P(out2), P(bias), P(dout), P(rs), P(pack), _lib.stream(dev)),
                    "hicgat_tail_bwd_fused_rows")
            elif heads is None:
                _lib.check(self.lib.hicgat_tail_bwd_fused(
                    P(dcoords), M, P(Y1), P(st1), P(Y2), P(st2), P(y3), P(st3), *[P(t) for t in ts], P(dx), P(dY1),
                    P(dY2), P(dy3), *wsa, P(pack), _lib.stream(dev)), "hicgat_tail_bwd_fused")
            else:
                h = heads
                assert h.dout.shape == (M, 512) and h.dout.is_contiguous() and h.dxa.shape == (M, 1024)
                assert h.dxa.is_contiguous() and h.rs.shape == (M, 8) and h.rs.is_contiguous()
                _lib.check(self.lib.hicgat_tail_bwd_fused_heads(
                    P(dcoords), M, P(Y1), P(st1), P(Y2), P(st2), P(y3), P(st3), *[P(t) for t in ts], P(dY1), P(dY2),
                    P(dy3), *wsa, int(h.act), P(h.Y0), P(h.W), P(h.bias), P(h.dout), P(h.rs), P(h.dxa), P(pack),
                    _lib.stream(dev)), "hicgat_tail_bwd_fused_heads")
        return dx, dY1, dY2, dy3, ws

    def tail_waves(self):
        """Waves per workgroup of the fused tail kernels (hicgat_tail_bwd_waves)."""
        return int(self.lib.hicgat_tail_bwd_waves())

    def tail_partial_rows(self, M):
        """Rows of LayerNorm partials hicgat_tail_bwd_fused leaves per workspace: one per workgroup."""
        return -(-M // 16)

    def ln_workspace(self, W, device):
        return _lib.workspace(self.lib.hicgat_ln_relu_res_workspace_bytes(W), device)

    def ln_relu_res_bwd_params(self, W, dgamma, dbeta, ws, accumulate=False):
        _lib.check(self.lib.hicgat_ln_relu_res_bwd_params(W, P(dgamma), P(dbeta), int(accumulate), P(ws), ws.numel(),
                                                          _lib.stream(ws.device)), "hicgat_ln_relu_res_bwd_params")

    # -- a10 --------------------------------------------------------------------------------------
    def adam_table(self, flat, grad, m, v, n, b1, b2, eps, table, step_ctr, counted=False):
        with _timed("adam"):
            _lib.check(self.lib.hicgat_adam_step_table_ex(P(flat), P(grad), P(m), P(v), int(n), float(b1), float(b2),
                                                          float(eps), P(table), table.shape[0], P(step_ctr),
                                                          int(bool(counted)), _lib.stream(flat.device)),
                       "hicgat_adam_step_table_ex")

    def step_begin(self, grad, step_ctr=None, pack=None):
        """zero_grad of the flat gradient buffer + (step_ctr) the device step count's advance, one launch;
        ``pack`` = (W1c, W2c, Wh or None, buffer): the tail's packed weight copies in the same launch
        (hicgat_step_begin_pack)."""
        if pack is not None:
            W1c, W2c, Wh, buf = pack
            for t in (W1c, W2c) + ((Wh,) if Wh is not None else ()):
                assert t.is_contiguous() and t.dtype == torch.float32
            n = int(self.lib.hicgat_tail_pack_bytes())
            assert buf.numel() * buf.element_size() >= n
            _lib.check(self.lib.hicgat_step_begin_pack(P(grad), grad.numel(), P(step_ctr), P(W1c), P(W2c), P(Wh), P(buf),
                                                       n, _lib.stream(grad.device)), "hicgat_step_begin_pack")
            return
        _lib.check(self.lib.hicgat_step_begin(P(grad), grad.numel(), P(step_ctr), _lib.stream(grad.device)),
                   "hicgat_step_begin")

    def adam(self, flat, grad, m, v, n, lr, b1, b2, eps, step):
        with _timed("adam"):
            _lib.check(self.lib.hicgat_adam_step(P(flat), P(grad), P(m), P(v), int(n), float(lr), float(b1),
                                                 float(b2), float(eps), int(step), _lib.stream(flat.device)),
                       "hicgat_adam_step")


_default = None


def default():
    global _default
    if _default is None:
        _default = HipKernels()
    return _default
