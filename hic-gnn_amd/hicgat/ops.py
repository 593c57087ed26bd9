"""Autograd functions over the HIP kernels (the product compute path; no CPU fallback).

* ``gat_conv``        -- PyG 1.7.2 GATConv forward/backward (a2, a4, a5 and their backward).
* ``pairwise_dist``   -- torch.cdist(c, c, p=2) forward/backward (a7), D materialised.
* ``fused_dist_loss`` -- cdist + MSELoss (+ Pearson / combined loss value) fused (a7-a9), D never
                         materialised; returns the loss scalar and keeps the fp64 stats.
"""
import contextlib
import os
import threading

import torch

from . import _lib, kernels, streams


def _sink(p):
    """The parameter's own ``.grad`` when it is a view into ``FlatAdam``'s flat gradient buffer
    (marked ``_hicgat_grad_sink``): the backward kernels then ADD the gradient into it in place
    (accumulate epilogue) and return ``None`` to autograd, which saves one add kernel and one
    temporary per parameter.  Otherwise ``None`` (ordinary autograd accumulation)."""
    if p is not None and getattr(p, "_hicgat_grad_sink", False) and p.grad is not None:
        return p.grad
    return None


# ---- weight-gradient side stream ---------------------------------------------------------------
# The parameter-gradient kernels (split-K dW GEMMs, bias column sums, GAT param_grad) feed only the
# optimizer, never the next backward op, so inside ``overlapped_param_grads`` they are issued on a
# side stream that forks from the backward's stream and is joined back before anything reads the
# flat gradient buffer (Adam / the gradient all-reduce).  The MFMA-bound GEMMs then run beside the
# L2-bound aggregation backward instead of in series with it; in a captured step the fork and join
# are graph edges.  Only sink-bound gradients (``_sink``) go to the side stream -- a gradient that
# is returned to autograd is consumed on the backward's stream and must be produced there.
_SIDE = {"on": 0, "streams": {}, "mains": {}, "hold": [], "queue": [], "grouped": 0, "jobs": [], "no_big": 0}
_SIDE_LOCK = threading.Lock()
OVERLAP_DEFAULT = True
# The tail's parameter-gradient launches (split-K dW GEMMs with their bias sums, the LayerNorm
# dgamma/dbeta sums, bias column sums) are DEFERRED: queued, and issued by ``side_flush`` on the side
# stream beside the GAT source-side gather (forked after the gather-free row pass).  Issued as they
# come, a captured step's graph placed some of them in front of the aggregation backward on its
# queue (2.036 vs 2.060 ms per step).  Measured slower and removed: largest-first
# or small-first issue order, the big dW GEMMs on a stream of their own or on the backward's stream,
# lin_l's dW queued behind the side work, the GAT param_grad on a second side stream or split around
# the gather, the source pass in row chunks, two side lanes on one GPU.


# single-GPU step: parameter-gradient jobs of at least this many multiply-adds (the first tail block's
# 512 x 512 dW, 5.2e9 at N = 20000) are held and issued with lin_l's dW as ONE grouped launch after
# the source gather (0: off -- they go to the side stream like the rest).  Round 4: 1.876 / 1.879 vs
# 1.889 / 1.888 ms per step with one side launch per item (profiles/r04i_ab_big_group.txt); with the
# side work as one grouped launch (SIDE_GROUPED) the big dW rides there: 0 since round 6
BIG_GROUP = float(os.environ.get("HICGAT_BIG_GROUP", "0"))


def side_begin():
    """Route sink-bound parameter gradients to the side stream until ``side_join``."""
    with _SIDE_LOCK:
        _SIDE["on"] += 1


def side_mark():
    """An event on the current stream marking where queued side work may start (``side_flush``)."""
    if not _SIDE["on"] or not _SIDE["queue"]:
        return None
    return streams.record()


_FLUSH_LANES = (0, 4, 5, 6)
SMALL_WORK = 4e6   # side_flush(lanes > 1): items below this many multiply-adds go first in their lane
# single-GPU step (one lane): the queued side work -- every dW / db / LayerNorm sum of the MLP tail,
# the first block's 512 x 512 dW included (BIG_GROUP 0) -- as ONE grouped weight-gradient + ONE
# grouped column-sum launch (hicgat_param_grads_grouped) beside the source gather, when every item has
# a job descriptor, instead of ~13 launches that each waited for room beside the gather; 0: one
# launch per item.  SIDE_GROUP_WGS: the grouped launch's workgroup target (the K split): fewer
# workgroups take fewer CUs from the gather; SIDE_SMALL_M 0: dense3's 3-row dW as an MFMA tile, not
# three 20 000-row weighted column sums (single-block chains, 157 µs of the side lane).  1.730-1.732
# vs 1.769-1.771 ms per step (profiles/r06rst_ab_side_grouped.txt, r06u_ab_side_grouped.txt)
SIDE_GROUPED = os.environ.get("HICGAT_SIDE_GROUPED", "1") != "0"
SIDE_GROUP_WGS = int(os.environ.get("HICGAT_SIDE_GROUP_WGS", "192"))
SIDE_SMALL_M = int(os.environ.get("HICGAT_SIDE_SMALL_M", "0"))


def side_flush(after=None, lanes=1):
    """Issue the queued parameter-gradient launches on the side stream, forked from the current
    stream at this point, or from the earlier point ``after`` (an event from ``side_mark``): the
    caller can then enqueue its own next kernel first, so a captured graph lists that kernel
    ahead of the side branch (they read only tensors produced before the fork point).

    ``lanes`` > 1 spreads the launches over that many side streams (largest work first, each to the
    least-loaded lane; every launch writes its own parameters' gradients, so they are independent):
    a rank's shard of the multi-GPU slab step has a gather window too short for the tail's queued
    launches in one chain.  The single-GPU step keeps one lane (a second one measured slower there,
    DESIGN section 7)."""
    with _SIDE_LOCK:
        queue, _SIDE["queue"] = _SIDE["queue"], []
    if not queue:
        return
    n = max(1, min(lanes, len(_FLUSH_LANES)))
    if n == 1 and SIDE_GROUPED and all(q[3] is not None for q in queue):
        with _side(*[t for _, keep, _, _ in queue for t in keep], after=after, lane=_FLUSH_LANES[0]):
            streams.stamp("side_begin")
            _grouped_launch(kernels.default(), [q[3] for q in queue], SIDE_GROUP_WGS, small_m=SIDE_SMALL_M)
            streams.stamp("side_end")
        return
    load, parts = [0] * n, [[] for _ in range(n)]
    if n == 1:
        parts[0] = queue                     # backward order
    else:
        for item in sorted(queue, key=lambda q: -q[2]):
            k = min(range(n), key=lambda a: (load[a], len(parts[a])))
            parts[k].append(item)
            load[k] += item[2]
    for lane, items in zip(_FLUSH_LANES, parts):
        if n > 1:
            # reductions without a GEMM (LayerNorm dgamma/dbeta sums: inputs ready, a few us each)
            # first in their lane, then the GEMMs
            items = [q for q in items if q[2] < SMALL_WORK] + [q for q in items if q[2] >= SMALL_WORK]
        if items:
            with _side(*[t for _, keep, _, _ in items for t in keep], after=after, lane=lane):
                streams.stamp("side_begin")
                for fn, _, _, _ in items:
                    fn()
                streams.stamp("side_end")


def side_record():
    """Events recorded now on every side stream in use: they complete when the side work issued
    so far (e.g. the tail's flushed dW GEMMs) has run.  [] when nothing went to a side stream."""
    if not _SIDE["on"]:
        return []
    with _SIDE_LOCK:
        sides = [_SIDE["streams"][key] for key in _SIDE["mains"]]
    return [streams.record(st) for st in sides]


@contextlib.contextmanager
def grouped_param_grads():
    """Inside: the sink-bound parameter gradients that have a job descriptor (every dW / db / LayerNorm
    sum of the Linear, dual-Linear and fused-tail backward) are collected instead of launched;
    ``grouped_flush`` then issues ALL of them as two launches (hicgat_param_grads_grouped).  A rank's
    share of the sharded step is too small for ~15 separate launches: queued over side lanes they
    were the critical path after the edge pass (profiles/r03w_simprof_xagg_P8_rank0_timeline.txt)."""
    with _SIDE_LOCK:
        _SIDE["grouped"] += 1
    try:
        yield
    except BaseException:
        # a failed backward: drop the collected descriptors, so no later grouped_flush adds this
        # step's partial dW / db into another step's gradient
        with _SIDE_LOCK:
            _SIDE["jobs"].clear()
        raise
    finally:
        with _SIDE_LOCK:
            _SIDE["grouped"] -= 1


def grouped_flush(K=None, extra=(), target_wgs=None, small_m=None):
    """Issue the collected jobs (plus ``extra`` descriptors) on the current stream: one grouped
    weight-gradient launch and one grouped column-sum launch.  Returns the tensors they read (the
    caller keeps them alive until the launches are ordered before any reuse)."""
    with _SIDE_LOCK:
        jobs, _SIDE["jobs"] = _SIDE["jobs"], []
    jobs = jobs + [(j, ()) for j in extra]
    if not jobs:
        return []
    _grouped_launch(K if K is not None else kernels.default(), [j for j, _ in jobs], target_wgs, small_m)
    return [t for _, keep in jobs for t in keep]


def _grouped_launch(K, descs, target_wgs=None, small_m=None):
    """descriptors: ("w", dy, x, dW, db[, accumulate]) / ("c", src, dst[, accumulate[, row weights]]);
    accumulate defaults on; a 2-D dst [segs, cols] takes the rows' sum in segments
    (kernels.param_grads_grouped)"""
    w = [(j[1], j[2], j[3], j[4], j[5] if len(j) > 5 else True) for j in descs if j[0] == "w"]
    c = [(j[1], j[2], j[3] if len(j) > 3 else True) + ((j[4],) if len(j) > 4 else ()) for j in descs
         if j[0] == "c"]
    K.param_grads_grouped(w, c, target_wgs, small_m)


def side_join():
    """Flush the queue, make every stream that forked work onto the side stream wait for it, and
    drop the held inputs.  Always runs the queued launches, even after an exception upstream, so
    no gradient kernel is left behind for a later step."""
    try:
        side_flush()
        if _SIDE["jobs"] and not _SIDE["grouped"]:
            # held big jobs that no GATConv backward issued (BIG_GROUP with another model): now
            _SIDE["hold"].extend(grouped_flush())
    finally:
        with _SIDE_LOCK:
            _SIDE["on"] = max(0, _SIDE["on"] - 1)
            for key, main in _SIDE["mains"].items():
                streams.join(main, _SIDE["streams"][key])
            _SIDE["mains"].clear()
            _SIDE["hold"].clear()


@contextlib.contextmanager
def overlapped_param_grads(enabled=None, hold_big=True):
    """``with overlapped_param_grads(): loss.backward()`` -- parameter gradients overlap the rest
    of the backward and are complete (ordered before the caller's stream) on exit.

    ``hold_big=False``: no BIG_GROUP holding -- for a backward that has no ``_GATConvFn`` to issue
    the held jobs with lin_l's dW (the sharded step runs the GATConv backward itself; a held job
    would otherwise be issued by ``side_join`` on the main stream, after the caller recorded the
    side streams' completion for its gradient all-reduce)."""
    if not (OVERLAP_DEFAULT if enabled is None else enabled):
        yield
        return
    side_begin()
    if not hold_big:
        with _SIDE_LOCK:
            _SIDE["no_big"] += 1
    try:
        yield
    finally:
        try:
            side_join()
        finally:
            if not hold_big:
                with _SIDE_LOCK:
                    _SIDE["no_big"] -= 1


def _param_launch(fn, *keep, small=False, work=0, job=None):
    """Launch a sink-bound parameter-gradient kernel ``fn()``: now on the current stream when not
    overlapping; queued for ``side_flush`` when deferring (``work``: its size, the issue order);
    else now on the side stream.  ``keep`` are the tensors ``fn`` reads (held until the join).
    ``job``: the same work as a descriptor for ``grouped_flush`` -- ("w", dy, x, dW, db) for
    dW += dy^T x (and db += column sums of dy), ("c", src, dst) for dst += column sums of src."""
    if job is not None and (_SIDE["grouped"] or (BIG_GROUP > 0 and _SIDE["on"] and not _SIDE["no_big"]
                                                 and work >= BIG_GROUP)):
        with _SIDE_LOCK:
            _SIDE["jobs"].append((job, keep))
        return
    if not _SIDE["on"]:
        fn()
    else:
        with _SIDE_LOCK:
            _SIDE["queue"].append((fn, keep, work, job))


def _side(*keep, after=None, lane=0):
    """Stream context for a sink-bound gradient kernel: side stream ``lane`` (after a fork from the
    current stream, or from the event ``after``) while overlapping, else a no-op.  ``keep`` are
    the inputs the side kernels read; they stay referenced until the join so the caching
    allocator cannot hand their memory to a later backward kernel while the side stream still
    reads it."""
    if not _SIDE["on"]:
        return contextlib.nullcontext()
    cur = torch.cuda.current_stream()
    dev = cur.device
    key = (dev, lane)
    with _SIDE_LOCK:
        side = _SIDE["streams"].get(key)
        if side is None:
            side = _SIDE["streams"][key] = streams.get(f"side{lane}", dev)
        _SIDE["mains"].setdefault(key, cur)
        _SIDE["hold"].extend(keep)
    if after is not None:
        streams.wait(side, after)
    else:
        streams.fork(side, cur)
    return torch.cuda.stream(side)


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.HicgatUnavailable("hicgat ops need CUDA (HIP) tensors; got a CPU tensor")


_ACTS = {None: 0, "relu": 1}
# the single-GPU GATConv's gather-free rows pass (hicgat_gat_agg_bwd_rows) in the one-kernel tail
# backward's epilogue when that tail consumes the layer's output (hicgat_tail_bwd_fused_rows); 0: the
# separate pass
FUSE_ROWS = os.environ.get("HICGAT_FUSE_ROWS", "1") != "0"
# the tail's weight pack written by the step's first launch (step_pack); 0: its own launch in the forward
STEP_PACK = os.environ.get("HICGAT_STEP_PACK", "1") != "0"


class _GATConvFn(torch.autograd.Function):
    """PyG 1.7.2 GATConv (+ an optional fused relu epilogue, act=1).  With gradients enabled the
    aggregation also emits out2 / S3 (include/hicgat.h), so the destination half of the backward
    is a streaming pass (``agg_bwd_rows``) and only the source half gathers."""

    @staticmethod
    def forward(ctx, x, W, att_l, att_r, bias, rowptr, col, negative_slope, act, tiles=None):
        _lib.lib()
        _dev_check(x, W, att_l, att_r, bias, rowptr, col)
        K = kernels.default()
        x = x.contiguous().float()
        W = W.contiguous()
        al = att_l.contiguous()
        ar = att_r.contiguous()
        N = x.shape[0]
        H = al.shape[-2]
        h, a_src, a_dst = K.linear_att(x, W, al, ar)
        D = h.shape[1]
        b = bias if bias is not None else torch.zeros(D, dtype=torch.float32, device=x.device)
        out = torch.empty((N, D), dtype=torch.float32, device=x.device)
        row_stats = torch.empty((N, 4 * H), dtype=torch.float32, device=x.device)
        train = any(ctx.needs_input_grad[:5])
        out2 = torch.empty((N, D), dtype=torch.float32, device=x.device) if train else None
        if tiles is not None:
            K.agg_fwd_tiled(rowptr, col, tiles, h, a_src, a_dst, b, negative_slope, act, out, out2, row_stats)
        else:
            K.agg_fwd_act(rowptr, col, 0, N, h, a_src, a_dst, b, negative_slope, act, out, out2, row_stats)
        ctx.tiles = tiles
        ctx.rows_state = None
        if train:
            ctx.save_for_backward(x, W, al, ar, h, a_src, a_dst, row_stats, rowptr, col, out, out2, b)
            if FUSE_ROWS:
                # the one-kernel tail that consumes ``out`` may run this layer's rows pass in its
                # backward's epilogue (_FusedTailFn; hicgat_tail_bwd_fused_rows): it finds these
                # operands on ``out`` and records the dout it wrote in the shared state
                ctx.rows_state = {"dout": None}
                out._hicgat_rows = (act, out2, row_stats, b, ctx.rows_state)
        ctx.has_bias = bias is not None
        ctx.ns = float(negative_slope)
        ctx.act = act
        ctx.params = (W, att_l, att_r, bias)
        return out

    @staticmethod
    def backward(ctx, dout):
        K = kernels.default()
        x, W, al, ar, h, a_src, a_dst, row_stats, rowptr, col, out, out2, b = ctx.saved_tensors
        N = x.shape[0]
        H = al.shape[-2]
        fused = ctx.rows_state is not None and ctx.rows_state["dout"] is not None
        if fused:
            # the tail's backward ran this layer's rows pass: dout (relu'd) and row_stats[:, 4:8] are
            # written, and the gradient that reached us must be exactly the dout it returned (a second
            # consumer of ``out`` would have added into it: then the rows pass saw only a part)
            if dout.data_ptr() != ctx.rows_state["dout"].data_ptr():
                raise RuntimeError("the GATConv output fed more than the fused tail: its rows pass was fused "
                                   "into the tail's backward (set HICGAT_FUSE_ROWS=0 for such a model)")
            ctx.rows_state["dout"] = None
        elif ctx.act:
            g, dout = dout.contiguous(), torch.empty_like(dout)
            K.agg_bwd_rows(0, N, ctx.act, g, out, b, out2, dout, row_stats)
        else:
            dout = dout.contiguous()
            K.agg_bwd_rows(0, N, 0, dout, out, b, out2, None, row_stats)
        fork = side_mark()   # the tail's queued dW / db launches run beside the source pass below
        dh = torch.empty_like(h)
        da_src = torch.empty_like(a_src)
        pW, pl, pr, pb = ctx.params
        sinks = (_sink(pl), _sink(pr), _sink(pb) if ctx.has_bias else None)
        use_sinks = all(t is not None for t in sinks)
        if ctx.tiles is not None:
            K.agg_bwd_src_tiled(ctx.tiles, h, a_src, a_dst, row_stats, dout, al, ar, ctx.ns, dh, da_src)
        else:
            streams.stamp("src_begin")
            K.agg_bwd_src(rowptr, col, 0, N, h, a_src, a_dst, row_stats, dout, al, ar, ctx.ns, dh, da_src)
            streams.stamp("src_end")
        side_flush(after=fork)
        # after the gathers: the GAT column sums, then lin_l's dW on this stream (with the held
        # first-block dW: BIG_GROUP).  The column sums on a side stream beside the grouped dW launch:
        # 1.964 / 1.970 vs 1.877 / 1.872 ms per step (profiles/r04l_ab_single_gpu.txt)
        if use_sinks:
            K.param_grad(h, dout, da_src, row_stats, H, out=(sinks[0].view(-1), sinks[1].view(-1), sinks[2]),
                         accumulate=True)
            datt_l = datt_r = dbias = None
        else:
            datt_l, datt_r, dbias = K.param_grad(h, dout, da_src, row_stats, H)
            datt_l, datt_r = datt_l.view(al.shape), datt_r.view(ar.shape)
            dbias = dbias if ctx.has_bias else None
        dW = None
        if ctx.needs_input_grad[1]:
            gW = _sink(pW)
            if gW is not None and _SIDE["jobs"]:
                # the held big dW jobs and lin_l's as one grouped launch (BIG_GROUP)
                _SIDE["hold"].extend(grouped_flush(K, [("w", dh, x, gW, None)]))
            else:
                dW = weight_grad(K, dh, x, out=gW, accumulate=gW is not None)
                if gW is not None:
                    dW = None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(0, 1, N, x.shape[1], h.shape[1], dh, W, torch.empty_like(x), name="gemm_dx")
        return (dx, dW, datt_l, datt_r, dbias, None, None, None, None, None)


# target workgroups of a split-K weight-gradient GEMM.  Alone, 512 measured best at N = 20000 (0.094
# vs 0.108 ms for 512x512x20000 at 1024, fewer fp32 slabs to add; profiles/r01_kbench_x3_sliced.txt);
# in the step, where the big dW GEMMs run two at a time beside each other after the source pass,
# 256 (half the slabs to add) is faster: 1.927 vs 1.942 ms per step, three A/B rounds
# (profiles/r02d_ab_step.txt)
_DW_BLOCKS = int(os.environ.get("HICGAT_DW_BLOCKS", "256"))


def _splits(m, n, k, target=None):
    """K-split for a weight-gradient GEMM whose K is the node count: enough workgroups to fill
    the 256 CUs, each split at least 256 rows deep."""
    target = _DW_BLOCKS if target is None else target
    bm = 128 if (m >= 128 and n >= 128) else 64
    tiles = -(-m // bm) * -(-n // bm)
    return max(1, min(k // 256, target // tiles))


def weight_grad(K, dy, x, out=None, accumulate=False, impl=None):
    """dW = dy^T x (Linear / lin_l weight gradient), K = rows, split-K MFMA GEMM."""
    rows, m = dy.shape
    n = x.shape[1]
    if out is None:
        out = torch.empty((m, n), dtype=torch.float32, device=dy.device)
    return K.gemm(1, 1, m, n, rows, dy, x, out, accumulate=accumulate, splits=_splits(m, n, rows), name="gemm_dw",
                  impl=impl)


def _weight_grad_to(K, p, dy, x):
    """dW = dy^T x into the parameter's sink (returns None) or a new tensor (returned)."""
    g = _sink(p)
    if g is not None:
        _param_launch(lambda: weight_grad(K, dy, x, out=g, accumulate=True), dy, x,
                      work=dy.shape[0] * dy.shape[1] * x.shape[1], job=("w", dy, x, g, None))
        return None
    return weight_grad(K, dy, x)


def _wb_grad_to(K, pW, pb, dy, x, need_w=True, need_b=True):
    """A Linear's dW = dy^T x and db = column sums of dy: ONE fp32 GEMM launch computes both
    (``hicgat_gemm_wgrad``, db from the staged dY tiles).  Into the parameters' sinks (returns
    (None, None); on the side stream when overlapping) or new tensors (returned).  Falls back to
    separate GEMM / column-sum launches when only one of the two is wanted, when the sinks are
    mixed."""
    need_b = need_b and pb is not None
    if not need_w:
        dW = _weight_grad_to(K, pW, dy, x) if need_w else None
        db = _bias_grad_to(K, pb, dy) if need_b else None
        return dW, db
    gW = _sink(pW)
    gb = _sink(pb) if need_b else None
    rows, m = dy.shape
    n = x.shape[1]
    sp = _splits(m, n, rows)
    if gW is not None and (gb is not None or not need_b):
        _param_launch(lambda: K.wgrad(dy, x, gW, gb, accumulate=True, splits=sp), dy, x, work=rows * m * n,
                      job=("w", dy, x, gW, gb))
        return None, None
    if gW is None and (not need_b or _sink(pb) is None):
        dW = torch.empty((m, n), dtype=torch.float32, device=dy.device)
        db = torch.empty(m, dtype=torch.float32, device=dy.device) if need_b else None
        K.wgrad(dy, x, dW, db, splits=sp)
        return dW, db
    return _weight_grad_to(K, pW, dy, x), _bias_grad_to(K, pb, dy)


def _bias_grad_to(K, p, dy):
    """db = column sums of dy into the parameter's sink (returns None) or a new tensor."""
    g = _sink(p)
    if g is not None:
        _param_launch(lambda: K.colsum(dy, g, accumulate=True), dy, small=True, job=("c", dy, g))
        return None
    return K.colsum(dy, torch.empty(dy.shape[1], dtype=torch.float32, device=dy.device))


class _LinearFn(torch.autograd.Function):
    """torch.nn.Linear (models.py:616-632 layers) forward/backward on the fp32 MFMA GEMM."""

    @staticmethod
    def forward(ctx, x, W, b):
        K = kernels.default()
        x = x.contiguous()
        M = x.shape[0]
        n_out, n_in = W.shape
        y = torch.empty((M, n_out), dtype=torch.float32, device=x.device)
        K.gemm(0, 0, M, n_out, n_in, x, W.contiguous(), y, bias=b, name="gemm_fwd")
        ctx.save_for_backward(x, W)
        ctx.has_bias = b is not None
        ctx.params = (W, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        K = kernels.default()
        x, W = ctx.saved_tensors
        dy = dy.contiguous()
        M = x.shape[0]
        n_out, n_in = W.shape
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(0, 1, M, n_in, n_out, dy, W.contiguous(), torch.empty_like(x), name="gemm_dx")
        dW, db = _wb_grad_to(K, ctx.params[0], ctx.params[1], dy, x, need_w=ctx.needs_input_grad[1],
                             need_b=ctx.has_bias and ctx.needs_input_grad[2])
        return dx, dW, db


def linear(x, W, b=None):
    """F.linear(x, W, b) on the MI355X GEMM kernels (CUDA tensors only)."""
    _dev_check(x, W, b)
    return _LinearFn.apply(x, W, b)


class _DualLinearFn(torch.autograd.Function):
    """Two Linear layers on the same input (models.py:638-639 / 646-647: dense* and align_dense*)
    as ONE GEMM over [W1; W2]: the input is read once; the backward adds both input gradients
    inside the GEMM (accumulate) instead of a separate add."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        K = kernels.default()
        x = x.contiguous()
        M = x.shape[0]
        n1, n2 = W1.shape[0], W2.shape[0]
        Wc = torch.cat([W1, W2]).contiguous()
        bc = torch.cat([b1, b2]).contiguous()
        Y = torch.empty((M, n1 + n2), dtype=torch.float32, device=x.device)
        K.gemm(0, 0, M, n1 + n2, x.shape[1], x, Wc, Y, bias=bc, name="gemm_fwd")
        ctx.save_for_backward(x, W1, W2)
        ctx.params = (W1, b1, W2, b2)
        return Y[:, :n1], Y[:, n1:]

    @staticmethod
    def backward(ctx, dy1, dy2):
        K = kernels.default()
        x, W1, W2 = ctx.saved_tensors
        M, n_in = x.shape
        dy1 = dy1.contiguous()
        dy2 = dy2.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(0, 1, M, n_in, W1.shape[0], dy1, W1, torch.empty_like(x), name="gemm_dx")
            K.gemm(0, 1, M, n_in, W2.shape[0], dy2, W2, dx, accumulate=True, name="gemm_dx")
        pW1, pb1, pW2, pb2 = ctx.params
        dW1, db1 = _wb_grad_to(K, pW1, pb1, dy1, x)
        dW2, db2 = _wb_grad_to(K, pW2, pb2, dy2, x)
        return dx, dW1, db1, dW2, db2


def dual_linear(x, lin1, lin2):
    _dev_check(x)
    return _DualLinearFn.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)


class _LnReluResFn(torch.autograd.Function):
    """relu(LayerNorm(y)) + res in one pass (models.py:641-655)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, res, eps):
        K = kernels.default()
        M, W = y.shape
        z = torch.empty((M, W), dtype=torch.float32, device=y.device)
        stats = torch.empty((M, 2), dtype=torch.float32, device=y.device)
        K.ln_relu_res_fwd(y, gamma, beta, eps, res, z, stats)
        ctx.save_for_backward(y, stats, gamma, beta)
        ctx.has_res = res is not None
        ctx.params = (gamma, beta)
        return z

    @staticmethod
    def backward(ctx, dz):
        K = kernels.default()
        y, stats, gamma, beta = ctx.saved_tensors
        dz = dz.contiguous()
        dy = torch.empty(y.shape, dtype=torch.float32, device=y.device)
        sg, sb = _sink(ctx.params[0]), _sink(ctx.params[1])
        if sg is not None and sb is not None and not _SIDE["on"]:
            K.ln_relu_res_bwd(dz, y, stats, gamma, beta, dy, sg, sb, accumulate=True)
            dgamma = dbeta = None
        elif sg is not None and sb is not None:
            ws = K.ln_workspace(y.shape[1], y.device)
            K.ln_relu_res_bwd(dz, y, stats, gamma, beta, dy, None, None, ws=ws)
            _param_launch(lambda: K.ln_relu_res_bwd_params(y.shape[1], sg, sb, ws, accumulate=True), ws)
            dgamma = dbeta = None
        else:
            dgamma = torch.empty_like(gamma)
            dbeta = torch.empty_like(beta)
            K.ln_relu_res_bwd(dz, y, stats, gamma, beta, dy, dgamma, dbeta)
        return dy, dgamma, dbeta, (dz if ctx.has_res else None), None


def ln_relu_res(y, norm, res=None):
    """F.relu(norm(y)) + res for a torch.nn.LayerNorm ``norm`` (elementwise affine)."""
    _dev_check(y)
    if y.stride(1) != 1:
        y = y.contiguous()
    if res is not None and res.stride(1) != 1:
        res = res.contiguous()
    return _LnReluResFn.apply(y, norm.weight, norm.bias, res, norm.eps)


def _adjacent(a, b):
    """``b`` starts right where ``a`` ends in the SAME storage (two views into FlatAdam's flat
    buffer): the pair is then one [a; b] tensor without a copy.  Two separate allocations that
    merely happen to sit back to back (the caching allocator packs small blocks into one segment)
    do not qualify: a view cannot span two storages."""
    return (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype
            and a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()
            and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size())


def _joined(a, b):
    """[a; b] along dim 0 -- a view when the two are adjacent (``flat_parameters`` order)."""
    if _adjacent(a, b):
        return torch.as_strided(a, (a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), a.stride())
    return torch.cat([a, b])


class _DualLnReluResFn(torch.autograd.Function):
    """relu(norm(lin1(x))) + lin2(x) -- the residual blocks of models.py:638-649 -- as
    ONE GEMM Y = x [W1; W2]^T + [b1; b2] and one row pass over Y = [y | res].  The backward's LN
    pass writes dY = [dy | dz] packed, so dx is ONE GEMM (K = 2W) and, with the pairs adjacent in
    FlatAdam's buffer (``flat_parameters``), dW and db are one GEMM / one column sum each."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2, gamma, beta, eps):
        K = kernels.default()
        x = x.contiguous()
        M = x.shape[0]
        w = W1.shape[0]
        Wc = _joined(W1, W2)
        bc = _joined(b1, b2)
        Y = torch.empty((M, 2 * w), dtype=torch.float32, device=x.device)
        K.gemm(0, 0, M, 2 * w, x.shape[1], x, Wc.contiguous(), Y, bias=bc.contiguous(), name="gemm_fwd")
        z = torch.empty((M, w), dtype=torch.float32, device=x.device)
        stats = torch.empty((M, 2), dtype=torch.float32, device=x.device)
        K.ln_relu_res_fwd(Y[:, :w], gamma, beta, eps, Y[:, w:], z, stats)
        ctx.save_for_backward(x, Y, stats, gamma, beta)
        ctx.params = (W1, b1, W2, b2, gamma, beta)
        return z

    @staticmethod
    def backward(ctx, dz):
        K = kernels.default()
        x, Y, stats, gamma, beta = ctx.saved_tensors
        W1, b1, W2, b2, pg, pb = ctx.params
        dz = dz.contiguous()
        M, w = dz.shape
        dY = torch.empty((M, 2 * w), dtype=torch.float32, device=dz.device)
        sg, sb = _sink(pg), _sink(pb)
        dgamma = dbeta = None
        if sg is not None and sb is not None and not _SIDE["on"]:
            K.ln_relu_res_bwd(dz, Y[:, :w], stats, gamma, beta, dY[:, :w], sg, sb, accumulate=True, dres=dY[:, w:])
        elif sg is not None and sb is not None:
            ws = K.ln_workspace(w, dz.device)
            K.ln_relu_res_bwd(dz, Y[:, :w], stats, gamma, beta, dY[:, :w], None, None, dres=dY[:, w:], ws=ws)
            _param_launch(lambda: K.ln_relu_res_bwd_params(w, sg, sb, ws, accumulate=True), ws)
        else:
            dgamma, dbeta = torch.empty_like(gamma), torch.empty_like(beta)
            K.ln_relu_res_bwd(dz, Y[:, :w], stats, gamma, beta, dY[:, :w], dgamma, dbeta, dres=dY[:, w:])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(0, 1, M, x.shape[1], 2 * w, dY, _joined(W1, W2).contiguous(), torch.empty_like(x),
                        name="gemm_dx")
        dW1, db1, dW2, db2 = _dual_param_grads(K, W1, b1, W2, b2, dY, x)
        return dx, dW1, db1, dW2, db2, dgamma, dbeta, None


def _dual_param_grads(K, W1, b1, W2, b2, dY, x):
    """dW / db of a dual-Linear pair from its packed output gradient dY = [dy1 | dy2] and input x:
    into the parameters' sinks (queued side work; returns Nones) or new tensors (returned)."""
    M, w = dY.shape[0], W1.shape[0]
    sW1, sW2, sb1, sb2 = _sink(W1), _sink(W2), _sink(b1), _sink(b2)
    dW1 = dW2 = db1 = db2 = None
    w_pair = sW1 is not None and sW2 is not None and _adjacent(sW1, sW2)
    b_pair = sb1 is not None and sb2 is not None and _adjacent(sb1, sb2)
    if w_pair and b_pair:
        # [dW1; dW2] and [db1; db2] of the pair in ONE GEMM launch (hicgat_gemm_wgrad)
        gWj, gbj, sp = _joined(sW1, sW2), _joined(sb1, sb2), _splits(2 * w, x.shape[1], M)
        _param_launch(lambda: K.wgrad(dY, x, gWj, gbj, accumulate=True, splits=sp), dY, x,
                      work=M * 2 * w * x.shape[1], job=("w", dY, x, gWj, gbj))
    else:
        if w_pair:
            gWj = _joined(sW1, sW2)
            _param_launch(lambda: weight_grad(K, dY, x, out=gWj, accumulate=True), dY, x,
                          job=("w", dY, x, gWj, None))
        else:
            dW1 = _weight_grad_to(K, W1, dY[:, :w], x)
            dW2 = _weight_grad_to(K, W2, dY[:, w:], x)
        if b_pair:
            gbj = _joined(sb1, sb2)
            _param_launch(lambda: K.colsum(dY, gbj, accumulate=True), dY, small=True, job=("c", dY, gbj))
        else:
            db1 = _bias_grad_to(K, b1, dY[:, :w].contiguous())
            db2 = _bias_grad_to(K, b2, dY[:, w:].contiguous())
    return dW1, db1, dW2, db2


def _ln_param_grads(K, gamma, beta, ws, rows):
    """A LayerNorm's dgamma / dbeta = the column sums of the first ``rows`` per-workgroup partial rows
    [dgamma | dbeta] that hicgat_tail_bwd_fused left in ``ws``: into the (adjacent) sinks as queued
    side work (ONE colsum launch over the live rows, its size as the lane-balancing work) or new
    tensors (returned)."""
    W = gamma.shape[0]
    part = ws.view(torch.float32)[:rows * 2 * W].view(rows, 2 * W)
    sg, sb = _sink(gamma), _sink(beta)
    if sg is not None and sb is not None and _adjacent(sg, sb):
        gj = _joined(sg, sb)
        _param_launch(lambda: K.colsum(part, gj, accumulate=True), ws, work=rows * 2 * W, job=("c", part, gj))
        return None, None
    out = K.colsum(part, torch.empty(2 * W, dtype=torch.float32, device=part.device))
    return out[:W], out[W:]


def dual_ln_relu_res(x, lin1, lin2, norm):
    """relu(norm(lin1(x))) + lin2(x) (models.py:638-641 / :646-649) on the fused kernels."""
    _dev_check(x)
    return _DualLnReluResFn.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias, norm.weight, norm.bias,
                                  norm.eps)


# The flagship's MLP tail forward as ONE launch (tail_fused.hip) for row counts in [MIN_M, MAX_M]
# (HICGAT_FUSED_TAIL=0: off).  Measured (profiles/r03r_ab_fused_tail.txt, 4-deep weight prefetch):
# a rank's shard at P = 8 (2 700 rows) 0.613 vs 0.650 ms per rank step, P = 4 (5 000) 0.877 vs
# 0.896, synth-2000 0.641 vs 0.664 ms per step; with the fused backward too (r03za) the P = 2 shard
# (10 000 rows) 1.302 / 1.307 vs 1.313 / 1.315 ms.  On the whole 20000-row graph it was slower
# (1.936 vs 1.913 ms per step) while its 16-row workgroups read the weights row-major -- a quarter
# of the load rate -- and is faster since they read packed copies (TAIL_PACK): 1.815 / 1.819 vs
# 1.871 / 1.876 ms per step (profiles/r05aa_fused_tail_20000_ab.txt), so MAX_M now covers it.
# Graphs below MIN_M (chr19: 58 / 114 loci) keep the per-layer kernels.
FUSED_TAIL = os.environ.get("HICGAT_FUSED_TAIL", "1") != "0"
FUSED_TAIL_MIN_M = int(os.environ.get("HICGAT_FUSED_TAIL_MIN_M", "1024"))
FUSED_TAIL_MAX_M = int(os.environ.get("HICGAT_FUSED_TAIL_MAX_M", "32768"))
# ... and its backward input-gradient chain in one launch too (tail_fused.hip; 0: the per-layer
# functions' backward steps on the fused forward's tensors): P = 8 rank step 0.583 vs 0.622 ms, P = 4
# 0.856 vs 0.889, synth-2000 0.628 vs 0.652 ms per step (profiles/r03t_ab_fused_tail_bwd.txt)
FUSED_TAIL_BWD = os.environ.get("HICGAT_FUSED_TAIL_BWD", "1") != "0"
# ... both reading W1c / W2c / the heads' W as packed copies (hicgat_tail_pack, one launch per
# forward; 0: the row-major weights)
TAIL_PACK = os.environ.get("HICGAT_TAIL_PACK", "1") != "0"


class _FusedTailFn(torch.autograd.Function):
    """models.py:638-659 after the relu (GATNetSelectiveResidualsUpdated.post_act): the forward in
    one kernel (hicgat_tail_fwd_fused), which writes the tensors the per-layer autograd functions
    would save; the backward runs those functions' own backward steps on them, in autograd's order
    (dense3, norm2, dense2, block 2, block 1), so its kernels, side-stream parameter gradients and
    sums are the per-layer path's."""

    @staticmethod
    def forward(ctx, x, Wa, ba, Wal, bal, ga, bea, W1, b1, W1al, b1al, g1, be1, W2, b2, g2, be2, W3, b3, eps,
                coords_out=None, heads=None, prepack=None):
        K = kernels.default()
        x = x.contiguous()
        W1c, b1c = _joined(Wa, Wal).contiguous(), _joined(ba, bal).contiguous()
        W2c, b2c = _joined(W1, W1al).contiguous(), _joined(b1, b1al).contiguous()
        # heads: x's rows are formed (written) by the kernel from the xagg GATConv's aggregates
        # the weights as packed copies for both kernels (made once per forward -- or by the training
        # step's first launch, ``prepack``: step_pack -- the backward reuses them)
        if prepack is not None:
            pack = prepack          # (heads: a pack with the heads' W, else the launch is refused)
        else:
            pack = K.tail_pack(W1c, W2c, heads.W if heads is not None else None) if TAIL_PACK else None
        coords, saved = K.tail_fwd_fused(x, W1c, b1c, ga.contiguous(), bea.contiguous(), W2c, b2c, g1.contiguous(),
                                         be1.contiguous(), W2.contiguous(), b2.contiguous(), g2.contiguous(),
                                         be2.contiguous(), W3.contiguous(), b3.contiguous(), eps, coords=coords_out,
                                         heads=heads, pack=pack)
        ctx.heads = heads
        ctx.pack = pack
        link = getattr(x, "_hicgat_rows", None) if heads is None else None
        # the GATConv's rows pass in this backward's epilogue: its relu output is exactly our input rows
        ctx.rows = link if (link is not None and FUSE_ROWS and K.tail_waves() == 16 and x.shape[1] == 512) else None
        if coords_out is not None:
            # the kernel wrote into the caller's buffer (e.g. the all-gather rows); the output is a
            # fresh tensor object over the same memory, so autograd sees a new output (no view or
            # in-place bookkeeping on the caller's buffer, which a collective then fills around it)
            coords = torch.empty(0, dtype=coords_out.dtype, device=coords_out.device).set_(
                coords_out.untyped_storage(), coords_out.storage_offset(), coords_out.shape, coords_out.stride())
        ctx.save_for_backward(x, *saved)
        ctx.params = (Wa, ba, Wal, bal, ga, bea, W1, b1, W1al, b1al, g1, be1, W2, b2, g2, be2, W3, b3)
        return coords

    @staticmethod
    def backward(ctx, dcoords):
        import types
        x, Y1, st1, z1, Y2, st2, z2, y3, st3, z3 = ctx.saved_tensors
        Wa, ba, Wal, bal, ga, bea, W1, b1, W1al, b1al, g1, be1, W2, b2, g2, be2, W3, b3 = ctx.params
        if FUSED_TAIL_BWD:
            # the input-gradient chain in one launch; the parameter gradients from its dY tensors
            # and LN partials, issued in the per-layer path's order (dense3, norm2, dense2, block 2,
            # block 1)
            K = kernels.default()
            dc = dcoords.contiguous()
            rows = None
            if ctx.rows is not None and ctx.needs_input_grad[0]:
                act, out2, rs, b, state = ctx.rows
                dout = torch.empty((dc.shape[0], 512), dtype=torch.float32, device=dc.device)
                rows = (act, x, out2, b, rs, dout)
            dx, dY1, dY2, dy3, (ws1, ws2, ws3) = K.tail_bwd_fused(
                dc, ctx.saved_tensors[1:], W3.contiguous(), W2.contiguous(), _joined(W1, W1al).contiguous(),
                _joined(Wa, Wal).contiguous(), ga.contiguous(), bea.contiguous(), g1.contiguous(), be1.contiguous(),
                g2.contiguous(), be2.contiguous(), heads=ctx.heads, pack=ctx.pack, rows=rows)
            if rows is not None:
                dx = dout               # the GATConv's backward finds it in the shared state and skips its rows pass
                state["dout"] = dout
            rows = K.tail_partial_rows(dc.shape[0])   # the kernel's partial rows: one per workgroup
            dW3, db3 = _wb_grad_to(K, W3, b3, dc, z3)
            dg2, dbe2 = _ln_param_grads(K, g2, be2, ws3, rows)
            dW2, db2 = _wb_grad_to(K, W2, b2, dy3, z2)
            dg1, dbe1 = _ln_param_grads(K, g1, be1, ws2, rows)
            dW1, db1, dW1al, db1al = _dual_param_grads(K, W1, b1, W1al, b1al, dY2, z1)
            dga, dbea = _ln_param_grads(K, ga, bea, ws1, rows)
            dWa, dba, dWal, dbal = _dual_param_grads(K, Wa, ba, Wal, bal, dY1, x)
            return (dx if ctx.needs_input_grad[0] else None, dWa, dba, dWal, dbal, dga, dbea, dW1, db1, dW1al, db1al,
                    dg1, dbe1, dW2, db2, dg2, dbe2, dW3, db3, None, None, None, None)
        T = (True,) * 8

        def c(**kw):
            return types.SimpleNamespace(needs_input_grad=T, **kw)

        dz3, dW3, db3 = _LinearFn.backward(c(saved_tensors=(z3, W3), params=(W3, b3), has_bias=True), dcoords)
        dy3, dg2, dbe2, _, _ = _LnReluResFn.backward(c(saved_tensors=(y3, st3, g2, be2), params=(g2, be2),
                                                       has_res=False), dz3)
        dz2, dW2, db2 = _LinearFn.backward(c(saved_tensors=(z2, W2), params=(W2, b2), has_bias=True), dy3)
        dz1, dW1, db1, dW1al, db1al, dg1, dbe1, _ = _DualLnReluResFn.backward(
            c(saved_tensors=(z1, Y2, st2, g1, be1), params=(W1, b1, W1al, b1al, g1, be1)), dz2)
        ctx1 = types.SimpleNamespace(needs_input_grad=(ctx.needs_input_grad[0],) + T[1:],
                                     saved_tensors=(x, Y1, st1, ga, bea), params=(Wa, ba, Wal, bal, ga, bea))
        dx, dWa, dba, dWal, dbal, dga, dbea, _ = _DualLnReluResFn.backward(ctx1, dz1)
        return (dx, dWa, dba, dWal, dbal, dga, dbea, dW1, db1, dW1al, db1al, dg1, dbe1, dW2, db2, dg2, dbe2,
                dW3, db3, None, None, None, None)


def fused_tail_ok(model, x):
    return (FUSED_TAIL and x.is_cuda and x.dim() == 2 and FUSED_TAIL_MIN_M <= x.shape[0] <= FUSED_TAIL_MAX_M
            and x.shape[1] == 512
            and x.dtype == torch.float32 and x.stride(1) == 1
            and model.norm_a.eps == model.norm1.eps == model.norm2.eps)


class TailHeads:
    """The xagg GATConv's operands of the head-fused tail kernels (hicgat_tail_{fwd,bwd}_fused_heads):
    X4 [2, 2, M, 512] (xa^h = X4[h, 0]), lin_l's weight W [512, 512] and bias [512], and the buffers
    they write: Y0 [M, 512] (the forward; the tail's input rows relu(Y0) go into ``fused_tail``'s x),
    dout [M, 512], the own rows' row stats rs [M, 8] and dxa [M, 1024] (the backward)."""

    def __init__(self, X4, W, bias, Y0, dout, rs, dxa, act=1):
        self.X4, self.W, self.bias, self.Y0, self.dout, self.rs, self.dxa, self.act = X4, W, bias, Y0, dout, rs, dxa, act


# HICGAT_TAIL_HEADS=0: the xagg step keeps its per-head GEMM launches, rows pass and dxa GEMMs
TAIL_HEADS = os.environ.get("HICGAT_TAIL_HEADS", "1") != "0"


def tail_heads_ok(model, x):
    return TAIL_HEADS and FUSED_TAIL_BWD and fused_tail_ok(model, x) and kernels.default().tail_waves() >= 8


def fused_tail(model, x, coords_out=None, heads=None):
    """GATNetSelectiveResidualsUpdated.post_act on the fused forward (``fused_tail_ok`` first);
    ``coords_out``: a contiguous [M, 3] buffer the coordinates are written into (and returned);
    ``heads`` (``TailHeads``, ``tail_heads_ok`` first): x's rows are formed from the xagg GATConv's
    aggregates in the same launch (x is written), and the backward writes the GATConv's dout /
    delta / dxa instead of x's gradient."""
    m = model
    return _FusedTailFn.apply(x, m.densea.weight, m.densea.bias, m.align_densea.weight, m.align_densea.bias,
                              m.norm_a.weight, m.norm_a.bias, m.dense1.weight, m.dense1.bias, m.align_dense1.weight,
                              m.align_dense1.bias, m.norm1.weight, m.norm1.bias, m.dense2.weight, m.dense2.bias,
                              m.norm2.weight, m.norm2.bias, m.dense3.weight, m.dense3.bias, m.norm_a.eps, coords_out,
                              heads, getattr(m, "_hicgat_prepack", None))


def step_pack(model, x):
    """The tail's packed weights as part of a training step's first launch: (W1c, W2c, None, buffer)
    for ``FlatAdam.zero_grad(pack=...)`` when the step's forward will run the one-kernel tail on x's
    N rows with packed weights (the flagship, ``fused_tail_ok``'s row range, the residual pairs
    adjacent in FlatAdam's buffer so [W; W_align] are views), else None.  The forward inside
    ``prepacked(model, job)`` then reads the buffer instead of packing again: one launch fewer per
    step (the weights change only at the previous step's Adam).  The sharded xagg step passes its
    own rows and hands the job to ``kernels.xagg_logits(pack=...)``, which adds lin_l's W (the
    head-fused tail's third weight)."""
    m = model
    if not (STEP_PACK and TAIL_PACK and FUSED_TAIL and x.is_cuda and hasattr(m, "align_densea") and hasattr(m, "norm_a")
            and FUSED_TAIL_MIN_M <= x.shape[0] <= FUSED_TAIL_MAX_M
            and m.norm_a.eps == m.norm1.eps == m.norm2.eps):
        return None
    if not (_adjacent(m.densea.weight, m.align_densea.weight) and _adjacent(m.dense1.weight, m.align_dense1.weight)):
        return None
    W1c, W2c = _joined(m.densea.weight, m.align_densea.weight), _joined(m.dense1.weight, m.align_dense1.weight)
    buf = getattr(m, "_hicgat_pack_buf", None)
    if buf is None or buf.device != x.device:
        n = int(kernels.default().lib.hicgat_tail_pack_bytes())
        buf = m._hicgat_pack_buf = torch.empty(n // 4, dtype=torch.float32, device=x.device)
    return (W1c.detach(), W2c.detach(), None, buf)


@contextlib.contextmanager
def prepacked(model, job):
    """The forward inside reads the pack ``job`` (``step_pack``) wrote, if any."""
    if job is None:
        yield
        return
    model._hicgat_prepack = job[3]
    try:
        yield
    finally:
        model._hicgat_prepack = None


def gat_conv(x, W, att_l, att_r, bias, adj, negative_slope=0.2, act=None):
    """GATConv forward; ``act="relu"`` returns relu(GATConv(x)) with the relu fused."""
    if adj.rowptr32 is None or adj.rowptr32.device != x.device:
        adj.to(x.device)
    return _GATConvFn.apply(x, W, att_l, att_r, bias, adj.rowptr32, adj.col32, negative_slope, _ACTS[act],
                            adj.tiles())


class _PairDistFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords):
        _lib.lib()
        _dev_check(coords)
        c = coords.contiguous().float()
        ctx.save_for_backward(c)
        return kernels.default().pairdist_fwd(c)

    @staticmethod
    def backward(ctx, dD):
        (c,) = ctx.saved_tensors
        return kernels.default().pairdist_bwd(c, dD.contiguous().float())


def pairwise_dist(coords):
    """torch.cdist(coords, coords, p=2) on the GPU (models.py:661)."""
    return _PairDistFn.apply(coords)


class _FusedLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords, tbuf, n, loss_kind, tile_begin, tile_end, stats, support=None):
        c = coords.contiguous().float()
        dc = torch.empty_like(c)
        loss = torch.empty((), dtype=torch.float32, device=c.device)
        if support is not None:
            kernels.default().fused_loss_support(c, support, n, loss_kind, stats, loss, dc)
        else:
            kernels.default().fused_loss(c, tbuf, n, loss_kind, tile_begin, tile_end, stats, loss, dc)
        ctx.save_for_backward(dc)
        return loss

    @staticmethod
    def backward(ctx, gl):
        (dc,) = ctx.saved_tensors
        # seeded by backward_from_loss with its resident ones tensor, never written since (the
        # version counter catches an in-place change by a hook): d(loss) = 1 exactly
        if gl is _UNIT_SEEDS.get(gl.device) and gl._version == 0:
            return dc, None, None, None, None, None, None, None
        return dc * gl, None, None, None, None, None, None, None


# loss.backward() fills a fresh ones tensor and the loss node then multiplies dcoords by it: two
# launches per step.  backward_from_loss seeds with one resident ones tensor per device instead, which
# the loss node recognises by identity AND an unchanged version counter (any in-place write to it --
# e.g. by a gradient hook -- bumps ``_version``, and the node then multiplies as usual) and skips
# the multiply -- the same bits.
_UNIT_SEEDS = {}


def backward_from_loss(loss):
    """``loss.backward()`` for a scalar loss from ``fused_dist_loss``, without the seed fill and the
    dcoords scaling launches."""
    seed = _UNIT_SEEDS.get(loss.device)
    if seed is None or seed.dtype != loss.dtype or seed._version != 0:
        seed = _UNIT_SEEDS[loss.device] = torch.ones((), dtype=loss.dtype, device=loss.device)
    torch.autograd.backward(loss, grad_tensors=seed)


LOSS_KINDS = {"mse": 0, "combined": 1, "contrastive": 2}   # include/hicgat.h loss_kind


def fused_dist_loss(coords, truth, kind="mse", tile_range=(0, -1), stats=None):
    """MSE(cdist(coords), truth) [kind="mse", HiC-GNN_main.py:127],
    MSE + alpha*(1 - pearson) [kind="combined", HiC_GAT_generalize_directly.py:219-225] with the
    gradient of the MSE only (the Pearson term is a detached host value in the reference), or
    0.1 * mean_{i<j} |T_ij - D_ij| [kind="contrastive", train_and_test_same_res_GAT_node2vec.py:107-134:
    differentiable; its fp64 value in stats[10], the returned scalar is its fp32 rounding].

    ``truth`` is a ``graph.Truth`` (stored symmetric; an asymmetric target is folded into the
    equivalent symmetric form there); with a background + support form (``truth.support``, e.g.
    cont2dist's target) the whole-matrix loss reads no truth in its O(N^2) pass.  ``stats`` (float64 [12], device) receives the moments, mse,
    r, alpha and total (see include/hicgat.h)."""
    _lib.lib()
    _dev_check(coords)
    if stats is None:
        stats = torch.empty(12, dtype=torch.float64, device=coords.device)
    kind_i = LOSS_KINDS[kind]
    if kind == "contrastive":
        truth = truth.upper()       # the contrastive loss reads truth[triu] as given
    t0, t1 = int(tile_range[0]), int(tile_range[1])
    # the background + support form (no truth stream) when the truth has one and all tiles are wanted
    whole = t0 == 0 and t1 in (-1, kernels.default().num_tiles(truth.n))
    support = getattr(truth, "support", None) if whole else None
    loss = _FusedLossFn.apply(coords, truth.buf, truth.n, kind_i, t0, t1, stats, support)
    return loss, stats


class _SageConvFn(torch.autograd.Function):
    """SAGEConv.forward (layers.py:55-77) on the HIP path: one wave-per-row pass writes
    z = [N_adj x | trunc(x)] and lin_l + lin_r run as ONE GEMM over [W_l | W_r] (K = 2F).  The
    x.long() branch carries no gradient (as in the reference); d x = N_adj^T (d out W_l)."""

    @staticmethod
    def forward(ctx, x, W_l, b_l, W_r, rowptr, col, w, inv_deg):
        K = kernels.default()
        x = x.contiguous().float()
        N, F = x.shape
        root = W_r is not None
        z = torch.empty((N, 2 * F if root else F), dtype=torch.float32, device=x.device)
        K.sage_agg(rowptr, col, w, inv_deg, 0, N, x, z, transpose=False, write_trunc=root)
        Wc = torch.cat([W_l, W_r], dim=1).contiguous() if root else W_l.contiguous()
        out = torch.empty((N, W_l.shape[0]), dtype=torch.float32, device=x.device)
        K.gemm(0, 0, N, W_l.shape[0], z.shape[1], z, Wc, out, bias=b_l, name="gemm_fwd")
        ctx.save_for_backward(z, W_l, rowptr, col, w, inv_deg)
        ctx.dims = (N, F, root, b_l is not None)
        ctx.params = (W_l, b_l, W_r)
        return out

    @staticmethod
    def backward(ctx, dout):
        K = kernels.default()
        z, W_l, rowptr, col, w, inv_deg = ctx.saved_tensors
        N, F, root, has_b = ctx.dims
        dout = dout.contiguous()
        dx = dWl = db = dWr = None
        pWl, pbl, pWr = ctx.params
        dWl, db = _wb_grad_to(K, pWl, pbl, dout, z[:, :F], need_w=ctx.needs_input_grad[1],
                              need_b=has_b and ctx.needs_input_grad[2])
        if root and ctx.needs_input_grad[3]:
            dWr = _weight_grad_to(K, pWr, dout, z[:, F:])
        if ctx.needs_input_grad[0]:
            dagg = K.gemm(0, 1, N, F, dout.shape[1], dout, W_l.contiguous(),
                          torch.empty((N, F), dtype=torch.float32, device=dout.device), name="gemm_dx")
            dx = K.sage_agg(rowptr, col, w, inv_deg, 0, N, dagg, torch.empty_like(dagg), transpose=True)
        return dx, dWl, db, dWr, None, None, None, None


def sage_conv(x, W_l, b_l, W_r, adj):
    """SAGEConv (layers.py:12-79) over a ``hicgat.Adj`` that carries ``value32``/``inv_deg``."""
    _dev_check(x, W_l, b_l, W_r)
    if adj.value32 is None or adj.inv_deg is None:
        raise ValueError("SAGEConv needs the edge weights: build the Adj with values (load_input / "
                         "Adj.from_dense_device / Adj(row, col, value).to(device))")
    return _SageConvFn.apply(x, W_l, b_l, W_r, adj.rowptr32, adj.col32, adj.value32, adj.inv_deg)
