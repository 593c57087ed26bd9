"""Destination-row sharded training step over P ranks (one GPU each, RCCL over xGMI).

BASELINE.json north star: "partition across the 8 GPUs of one node by sharding destination nodes
with an RCCL all-gather of the 512-d node embeddings"; SURVEY.md section 8(e).  The reference is
single-process (no collectives anywhere), so every exchange below is new.

Partition (``ShardPlan``):
  * destination rows in P contiguous blocks balanced by nnz -- bounds from a prefix sum over
    rowptr (the CSR's own rowptr IS that prefix sum), so a dense Hi-C band and a sparse tail get
    the same edge count per rank;
  * every node buffer is [P*R, .] with R = the largest block: rank p's rows sit at buffer rows
    p*R .. p*R + n_p - 1 (padding after them), so each all-gather is one in-place equal-chunk
    ``all_gather_into_tensor``.  Global row g lives at buffer row ``gidx[g]``;
  * each rank holds ONLY its rows of the graph (a padded rowptr whose other rows are empty, its
    edges with columns remapped to buffer rows), its rows of x, and the band of the truth its
    share of the upper-triangle loss tiles reads (tile-rows I0..I1, columns from I0*128 on).

Per step:
  forward:  h_p = x_p W^T (MFMA) into its buffer rows -> all_gather(h) [P*R, 512]
            (``replicate_x=True``: the SURVEY 8(e) ablation -- every rank holds all of x and
            computes h for every row, no all-gather of h)
            logits for all rows from the gathered h; aggregation (+ relu, out2, S3) of own rows;
            MLP tail on own rows -> all_gather(coords) -> global order (one index_select)
            fused distance/MSE over this rank's tile range of its truth band
            one fp64 all_reduce of [loss moments | dcoords]; finalize the loss
  backward: tail backward on own rows -> GAT bwd rows pass (relu backward, delta, da_dst; no
            gather) -> one all_gather of packed rows [dout (512) | row stats (max, sum, delta,
            da_dst)] -> GAT source pass on own rows (dh complete: a row's CSR list is every row
            that lists it, the graph is symmetric) -> dW_p = dh_p^T x_p, datt / dbias partials
            -> all_reduce(one flat fp32 grad buffer) -> identical Adam on every rank.
Strong scaling: the step is the same whole-graph step as on one GPU; results equal the 1-GPU
step up to the summation order of the all-reduces (tests/test_dist_gloo.py).

The trainer only talks to a kernel object (``hicgat.kernels.HipKernels`` in production), so the
partitioning and collectives are testable on CPU with gloo and a torch stand-in.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import ops
from .ops import _ACTS, weight_grad
from .optim import FlatAdam

TILE = 128


def partition_rows(rowptr, P):
    """Contiguous destination-row blocks with ~nnz/P CSR entries each: bounds [P+1], block p =
    rows [bounds[p], bounds[p+1]).  Boundary p is the row whose CSR start is nearest p*nnz/P."""
    rp = np.asarray(rowptr, dtype=np.int64)
    N = rp.shape[0] - 1
    nnz = int(rp[-1])
    b = np.zeros(P + 1, dtype=np.int64)
    b[P] = N
    for p in range(1, P):
        t = p * nnz / P
        r = int(np.searchsorted(rp, t, side="left"))     # first row whose start reaches t
        if r > 0 and (t - rp[r - 1]) < (rp[min(r, N)] - t):
            r -= 1
        b[p] = min(max(r, b[p - 1]), N)
    return b


def _tri_start(I, nb):
    return I * nb - I * (I - 1) // 2


def tri_row(t, nb):
    """Tile-row of upper-triangle tile ``t`` (row-major over I <= J), as the kernel decodes it."""
    lo, hi = 0, nb - 1
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if _tri_start(mid, nb) <= t:
            lo = mid
        else:
            hi = mid - 1
    return lo


class ShardPlan:
    """The static partition of a set_diag'd symmetric CSR (host int arrays) over P ranks."""

    def __init__(self, rowptr, col, P):
        rp = np.asarray(rowptr, dtype=np.int64)
        self.col = np.asarray(col, dtype=np.int64)
        self.rp = rp
        self.P = P
        self.N = N = rp.shape[0] - 1
        self.bounds = partition_rows(rp, P)
        self.counts = np.diff(self.bounds)
        self.R = R = max(1, int(self.counts.max()))
        owner = np.repeat(np.arange(P, dtype=np.int64), self.counts)
        self.gidx = owner * R + (np.arange(N, dtype=np.int64) - self.bounds[owner])
        self.nnz = np.array([rp[self.bounds[p + 1]] - rp[self.bounds[p]] for p in range(P)], dtype=np.int64)
        nb = (N + TILE - 1) // TILE
        self.tiles = nb * (nb + 1) // 2
        self.nb = nb

    def rows(self, rank):
        """(global first row, global end row, first buffer row)."""
        return int(self.bounds[rank]), int(self.bounds[rank + 1]), rank * self.R

    def local_csr(self, rank):
        """Padded rowptr [P*R + 1] (only this rank's buffer rows have edges) and its columns
        remapped to buffer rows (int32)."""
        r0, r1, q0 = self.rows(rank)
        e0, e1 = int(self.rp[r0]), int(self.rp[r1])
        rp = np.empty(self.P * self.R + 1, dtype=np.int64)
        rp[:q0 + 1] = 0
        rp[q0:q0 + (r1 - r0) + 1] = self.rp[r0:r1 + 1] - e0
        rp[q0 + (r1 - r0):] = e1 - e0
        return rp.astype(np.int32), self.gidx[self.col[e0:e1]].astype(np.int32)

    def tile_range(self, rank):
        """This rank's contiguous share of the upper-triangle loss tiles."""
        return self.tiles * rank // self.P, self.tiles * (rank + 1) // self.P

    def truth_band(self, rank):
        """(row0, row1, col0): the truth rows / first column the rank's tile range reads."""
        t0, t1 = self.tile_range(rank)
        if t1 <= t0:
            return 0, 0, 0
        I0, I1 = tri_row(t0, self.nb), tri_row(t1 - 1, self.nb)
        return I0 * TILE, min(self.N, (I1 + 1) * TILE), I0 * TILE


def _all_gather_inplace(buf, own, group):
    """All-gather where this rank's input ``own`` is its own chunk of ``buf`` (RCCL in place)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(buf, own, group=group)
    else:
        dist.all_gather(list(buf.chunk(dist.get_world_size(group))), own.clone(), group=group)


class ShardedTrainer:
    def __init__(self, model, x, adj, truth, lr=1e-3, kind="mse", group=None, kern=None, replicate_x=False):
        if kern is None:
            from .kernels import default
            kern = default()
        self.K = kern
        self.model = model
        self.group = group
        self.P = P = dist.get_world_size(group)
        self.rank = rank = dist.get_rank(group)
        self.kind = {"mse": 0, "combined": 1}[kind]
        self.replicate_x = bool(replicate_x)
        dev = model.conv.lin_l.weight.device
        N = x.shape[0]
        self.N = N
        plan = ShardPlan(adj.rowptr32.cpu().numpy(), adj.col32.cpu().numpy(), P)
        self.plan = plan
        R = plan.R
        self.R = R
        self.r0, self.r1, self.q0 = plan.rows(rank)
        self.local_rows = self.r1 - self.r0
        self.q1 = self.q0 + self.local_rows
        if self.local_rows == 0:
            raise ValueError(f"rank {rank} owns no rows (P = {P} > rows)")
        rp, cl = plan.local_csr(rank)
        self.rowptr = torch.from_numpy(rp).to(dev)
        self.col = torch.from_numpy(cl).to(dev)
        self.local_nnz = int(cl.shape[0])
        self.gidx = torch.from_numpy(plan.gidx).to(dev)
        conv = model.conv
        self.W, self.att_l, self.att_r, self.bias = conv.lin_l.weight, conv.att_l, conv.att_r, conv.bias
        self.ns = conv.negative_slope
        self.H = conv.heads
        self.D = D = conv.heads * conv.out_channels
        F = x.shape[1]
        f32 = dict(dtype=torch.float32, device=dev)
        self.x_loc = x[self.r0:self.r1].to(dev).contiguous().float()
        if self.replicate_x:
            self.x_pad = torch.zeros((P * R, F), **f32)
            self.x_pad[self.gidx] = x.to(dev).float()
        # the truth band of this rank's loss tiles (the full matrix is not kept)
        self.t0, self.t1 = plan.tile_range(rank)
        b0, b1, c0 = plan.truth_band(rank)
        self.trow0, self.tcol0 = b0, c0
        self.tband = truth.buf[b0:b1, c0:].contiguous() if b1 > b0 else torch.zeros((1, 4), **f32)
        # every [P*R, .] buffer: rank p's rows are the p-th R-row chunk (in-place all-gathers)
        self.h = torch.zeros((P * R, D), **f32)
        self.out = torch.zeros((P * R, D), **f32)
        self.out2 = torch.zeros((P * R, D), **f32)
        self.gbuf = torch.zeros((P * R, D), **f32)
        self.act = _ACTS[getattr(model, "conv_act", None)]
        # packed rows [dout (D) | row stats (4H)]: one all-gather carries both to the source pass
        self.pack = torch.zeros((P * R, D + 4 * self.H), **f32)
        self.dh = torch.zeros((P * R, D), **f32)
        self.da_src = torch.zeros((P * R, self.H), **f32)
        self.rs = torch.zeros((P * R, 4 * self.H), **f32)
        self.coords_buf = torch.zeros((P * R, 3), **f32)
        self.dcoords = torch.zeros((N, 3), **f32)
        # one fp64 all-reduce for the loss moments (7) and dcoords (3N)
        self.red = torch.zeros(7 + 3 * N, dtype=torch.float64, device=dev)
        self.stats = torch.zeros(12, dtype=torch.float64, device=dev)
        self.loss = torch.zeros((), **f32)
        self.opt = FlatAdam(model.flat_parameters(), lr=lr, kern=kern)

    def captured(self, warmup=2):
        """The step as one hipGraph (kernels + RCCL collectives, "nccl" backend only): one replay
        per step removes the ~70 host launches that would otherwise bound a small per-rank shard.
        The ``warmup`` eager steps are real training steps."""
        from .graphs import CapturedStep
        if dist.get_backend(self.group) != "nccl":
            raise RuntimeError("graph capture of the sharded step needs the nccl (RCCL) backend")
        if getattr(self.opt, "step_ctr", None) is None:
            self.opt.enable_device_step()
        return CapturedStep(self.step, warmup=warmup)

    def _own(self, buf):
        return buf[self.q0:self.q0 + self.R]

    def step(self):
        K, g, q0, q1, N, D = self.K, self.group, self.q0, self.q1, self.N, self.D
        self.opt.zero_grad()
        self.model.train()
        W, al, ar = self.W.detach(), self.att_l.detach(), self.att_r.detach()
        # ---- forward ------------------------------------------------------------------------
        if self.replicate_x:
            _, a_src, a_dst = K.linear_att(self.x_pad, W, al, ar, h=self.h)
        else:
            K.linear_att(self.x_loc, W, al, ar, h=self.h[q0:q1])
            _all_gather_inplace(self.h, self._own(self.h), g)
            a_src, a_dst = K.att_logits(self.h, al, ar)
        K.agg_fwd_act(self.rowptr, self.col, q0, q1, self.h, a_src, a_dst, self.bias.detach(), self.ns, self.act,
                      self.out, self.out2, self.rs)
        o = self.out[q0:q1].detach().requires_grad_(True)
        coords_loc = self.model.post_act(o) if self.act else self.model.tail(o)
        self.coords_buf[q0:q1].copy_(coords_loc.detach())
        _all_gather_inplace(self.coords_buf, self._own(self.coords_buf), g)
        coords = self.coords_buf.index_select(0, self.gidx)
        K.fused_loss(coords, self.tband, N, self.kind, self.t0, self.t1, self.stats, self.loss, self.dcoords,
                     row0=self.trow0, col0=self.tcol0)
        self.red[:7].copy_(self.stats[:7])
        self.red[7:].copy_(self.dcoords.view(-1))
        dist.all_reduce(self.red, group=g)
        self.stats[:7].copy_(self.red[:7])
        self.dcoords.view(-1).copy_(self.red[7:])
        K.loss_finalize(N, self.kind, self.stats, self.loss)
        # ---- backward -----------------------------------------------------------------------
        # parameter gradients on the side stream from here to the gradient all-reduce (ops.py)
        with ops.overlapped_param_grads(self.x_loc.is_cuda and ops.OVERLAP_DEFAULT):
            coords_loc.backward(self.dcoords[self.r0:self.r1])
            dout, rs_all = self.pack[:, :D], self.pack[:, D:]
            self.gbuf[q0:q1].copy_(o.grad)
            # act: writes dout = g * relu'(out) straight into the packed rows; otherwise dout is g
            K.agg_bwd_rows(q0, q1, self.act, self.gbuf, self.out, self.bias.detach(), self.out2, dout, self.rs)
            fork = ops.side_mark()   # the tail's queued dW / db launches run beside the all-gather + source pass
            if not self.act:
                dout[q0:q1].copy_(self.gbuf[q0:q1])
            rs_all[q0:q1].copy_(self.rs[q0:q1])
            _all_gather_inplace(self.pack, self._own(self.pack), g)
            K.agg_bwd_src(self.rowptr, self.col, q0, q1, self.h, a_src, a_dst, rs_all, dout, al, ar, self.ns,
                          self.dh, self.da_src)
            ops.side_flush(after=fork)
            dbias = self.bias.grad if self.bias is not None else torch.empty(D, device=self.h.device)
            with torch.no_grad():
                # lin_l's dW on the side stream (joined before the gradient all-reduce), param_grad
                # beside it on this stream
                with ops._side(self.dh, self.x_loc):
                    if self.x_loc.is_cuda:
                        weight_grad(K, self.dh[q0:q1], self.x_loc, out=self.W.grad, accumulate=True)
                    else:
                        self.W.grad.addmm_(self.dh[q0:q1].t(), self.x_loc)
            K.param_grad(self.h[q0:q1], dout[q0:q1].contiguous(), self.da_src[q0:q1], self.rs[q0:q1], self.H,
                         out=(self.att_l.grad.view(-1), self.att_r.grad.view(-1), dbias), accumulate=True)
        dist.all_reduce(self.opt.grad, group=g)
        self.opt.step()
        return self.loss, self.stats, coords
