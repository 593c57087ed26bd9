"""Destination-row sharded training step over P ranks (one GPU each, RCCL over xGMI).

BASELINE.json north star: "partition across the 8 GPUs of one node by sharding destination nodes
with an RCCL all-gather of the 512-d node embeddings".  The reference is single-process (SURVEY
section 2: no collectives anywhere), so every exchange below is new:

  rank p owns rows [p*R, min(N, (p+1)*R)), R = ceil(N/P) (contiguous, so the gathered buffers are
  in global row order: buffer row == global node id; the CSR, x and the truth are replicated).
  forward:  h_p = x_p W^T (MFMA, written into its rows of h) -> all_gather(h) in place
                                                                 [N, 512] fp32, 41 MB at N=20000
            a_src, a_dst for all rows from the gathered h (one cheap pass, no collective)
            GAT aggregation for own rows (+ the model's fused activation and the out2 / S3
            training outputs) -> MLP tail on own rows -> all_gather(coords) [N, 3]
            fused distance/MSE over this rank's share of the upper-triangle tiles
            one fp64 all_reduce of [loss moments | dcoords] ; finalize loss
  backward: tail backward on own rows -> GAT bwd rows pass (activation backward, delta, da_dst;
            no gather) -> one all_gather of packed rows [dout (512) | row stats (max, sum, delta,
            da_dst)]
            GAT bwd pass 2 on own rows -> dh_p (complete: own rows gather dout of all neighbours)
            dW_p = dh_p^T x_p, datt/dbias partial -> all_reduce(one flat fp32 grad buffer)
            identical Adam step on every rank (weights stay replicated).
Strong scaling: the step is the same whole-graph step as on one GPU; results equal the 1-GPU
step up to the summation order of the all-reduces (tests/test_dist_gloo.py).

The trainer only talks to a kernel object (``hicgat.kernels.HipKernels`` in production), so the
partitioning and collectives are testable on CPU with gloo and a torch stand-in.
"""
import torch
import torch.distributed as dist

from . import ops
from .ops import _ACTS, weight_grad
from .optim import FlatAdam


def _all_gather_inplace(buf, own, group):
    """All-gather where this rank's input ``own`` is its own chunk of ``buf`` (RCCL in place)."""
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(buf, own, group=group)
    else:
        dist.all_gather(list(buf.chunk(dist.get_world_size(group))), own.clone(), group=group)


class ShardedTrainer:
    def __init__(self, model, x, adj, truth, lr=1e-3, kind="mse", group=None, kern=None):
        if kern is None:
            from .kernels import default
            kern = default()
        self.K = kern
        self.model = model
        self.group = group
        self.P = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.kind = {"mse": 0, "combined": 1}[kind]
        N = x.shape[0]
        P = self.P
        R = (N + P - 1) // P
        self.N, self.R = N, R
        self.r0 = min(N, self.rank * R)
        self.r1 = min(N, self.r0 + R)
        self.local_rows = self.r1 - self.r0
        dev = x.device
        conv = model.conv
        self.W, self.att_l, self.att_r, self.bias = conv.lin_l.weight, conv.att_l, conv.att_r, conv.bias
        self.ns = conv.negative_slope
        self.H = conv.heads
        D = conv.heads * conv.out_channels
        self.x_loc = x[self.r0:self.r1].contiguous().float()
        self.rowptr, self.col = adj.rowptr32, adj.col32
        rp = self.rowptr
        self.local_nnz = int(rp[self.r1].item() - rp[self.r0].item())
        self.truth = truth
        f32 = dict(dtype=torch.float32, device=dev)
        self.D = D
        # every [P*R, .] buffer is in global row order; rank p's own rows are the p-th R-row chunk,
        # so the all-gathers run in place (no staging copies)
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
        self.coords = torch.zeros((P * R, 3), **f32)
        self.dcoords = torch.zeros((N, 3), **f32)
        # one fp64 all-reduce for the loss moments (7) and dcoords (3N)
        self.red = torch.zeros(7 + 3 * N, dtype=torch.float64, device=dev)
        self.stats = torch.zeros(12, dtype=torch.float64, device=dev)
        self.loss = torch.zeros((), **f32)
        T = kern.num_tiles(N)
        self.t0 = T * self.rank // P
        self.t1 = T * (self.rank + 1) // P
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
        return buf[self.rank * self.R:(self.rank + 1) * self.R]

    def step(self):
        K, g, r0, r1, N, D = self.K, self.group, self.r0, self.r1, self.N, self.D
        self.opt.zero_grad()
        self.model.train()
        # ---- forward ------------------------------------------------------------------------
        K.linear_att(self.x_loc, self.W.detach(), self.att_l.detach(), self.att_r.detach(), h=self.h[r0:r1])
        _all_gather_inplace(self.h, self._own(self.h), g)
        a_src, a_dst = K.att_logits(self.h, self.att_l.detach(), self.att_r.detach())
        K.agg_fwd_act(self.rowptr, self.col, r0, r1, self.h, a_src, a_dst, self.bias.detach(), self.ns, self.act,
                      self.out, self.out2, self.rs)
        o = self.out[r0:r1].detach().requires_grad_(True)
        coords_loc = self.model.post_act(o) if self.act else self.model.tail(o)
        self.coords[r0:r1].copy_(coords_loc.detach())
        _all_gather_inplace(self.coords, self._own(self.coords), g)
        coords = self.coords[:N]
        K.fused_loss(coords, self.truth.buf, N, self.kind, self.t0, self.t1, self.stats, self.loss, self.dcoords)
        self.red[:7].copy_(self.stats[:7])
        self.red[7:].copy_(self.dcoords.view(-1))
        dist.all_reduce(self.red, group=g)
        self.stats[:7].copy_(self.red[:7])
        self.dcoords.view(-1).copy_(self.red[7:])
        K.loss_finalize(N, self.kind, self.stats, self.loss)
        # ---- backward -----------------------------------------------------------------------
        # parameter gradients on the side stream from here to the gradient all-reduce (ops.py)
        overlap = self.x_loc.is_cuda and ops.OVERLAP_DEFAULT
        if overlap:
            ops.side_begin()
        coords_loc.backward(self.dcoords[r0:r1])
        dout, rs_all = self.pack[:, :D], self.pack[:, D:]
        self.gbuf[r0:r1].copy_(o.grad)
        # act: writes dout = g * relu'(out) straight into the packed rows; otherwise dout is g
        K.agg_bwd_rows(r0, r1, self.act, self.gbuf, self.out, self.bias.detach(), self.out2, dout, self.rs)
        if not self.act:
            dout[r0:r1].copy_(self.gbuf[r0:r1])
        rs_all[r0:r1].copy_(self.rs[r0:r1])
        _all_gather_inplace(self.pack, self._own(self.pack), g)
        K.agg_bwd_src(self.rowptr, self.col, r0, r1, self.h, a_src, a_dst, rs_all, dout,
                      self.att_l.detach(), self.att_r.detach(), self.ns, self.dh, self.da_src)
        dbias = self.bias.grad if self.bias is not None else torch.empty(D, device=self.h.device)
        K.param_grad(self.h[r0:r1], dout[r0:r1].contiguous(), self.da_src[r0:r1], self.rs[r0:r1], self.H,
                     out=(self.att_l.grad.view(-1), self.att_r.grad.view(-1), dbias), accumulate=True)
        with torch.no_grad():
            weight_grad(K, self.dh[r0:r1], self.x_loc, out=self.W.grad, accumulate=True) if self.x_loc.is_cuda \
                else self.W.grad.addmm_(self.dh[r0:r1].t(), self.x_loc)
        if overlap:
            ops.side_join()
        dist.all_reduce(self.opt.grad, group=g)
        self.opt.step()
        return self.loss, self.stats, coords
