"""Destination-row sharded training step over P ranks (one GPU each, RCCL over xGMI).

BASELINE.json north star: "partition across the 8 GPUs of one node by sharding destination nodes
with an RCCL all-gather of the 512-d node embeddings"; SURVEY.md section 8(e).  The reference is
single-process (no collectives anywhere), so every exchange below is new.

Partition (``ShardPlan``): destination rows in P contiguous blocks balanced by nnz (the CSR's own
rowptr is the prefix sum), every rank keeping at least one row; the upper-triangle loss tiles in P
contiguous ranges; the loss's support rows (the contact set of cont2dist's target) in P blocks
balanced by support nnz.

Three step forms (``mode``; "auto" picks xagg from P = 2, ``resolve_mode``):

``"slab"`` -- no per-step collective larger than the 2.4 MB gradient buffer.  The 512-d
  node embeddings x are constant, so they are all-gathered ONCE (every rank holds all of x, 41 MB)
  and each rank recomputes h = x W^T for every row (10.5 GFLOP, ~0.1 ms) instead of all-gathering
  h every step.  The backward's source side is split by DESTINATION owner instead of by source
  row: rank p runs the source pass over every row r but only over the neighbours i it owns (the
  "column slab" of the symmetric CSR: nnz/P entries), which needs only its own dout_i / row stats,
  so the [dout | stats] all-gather disappears too.  That yields a partial dh_r and da_src_r for
  every r; lin_l's dW = sum_r dh_r x_r^T and datt_src = sum_r da_src_r h_r are linear in them, so
  each rank forms its partial dW over all rows (x is replicated) and the ordinary gradient
  all-reduce sums the partials.  Per step: all-gather of coords (N x 3), one fp64 all-reduce of
  [loss moments | dcoords], the gradient all-reduce in two buckets -- the MLP tail's (ready when
  the side stream's dW GEMMs finish, reduced on a comm stream beside lin_l's dW GEMM) and the
  GATConv's -- and identical Adam on every rank.
``"xagg"`` (what "auto" runs) -- the aggregate-first GATConv (gat_xagg.hip): by linearity per head,
  out_i^h = W_h (sum_j alpha_ij x_j) + b^h, with a_src = x (W_h^T att^h); x is replicated (gathered
  once), every GEMM runs on the rank's own rows, the backward's edge pass folds the source side in
  (g = sum ds x, reduced as an 8 KB all-reduce; W's att (x) g term and datt applied to the summed g
  on every rank).  The tail's and the heads' dW and the flat-gradient all-reduce run on a side stream
  beside the edge pass.  Per step: coords all-gather, the fp64 [moments | dcoords] all-reduce, the
  flat-gradient all-reduce, g's all-reduce.
``"allgather"`` -- the north star's literal form: each rank computes h for its rows, RCCL
  all-gather of h [N, 512] before the layer; after the backward's row pass one all-gather of packed
  rows [dout | row stats] so each rank's source pass covers its own rows r completely (its dW is
  over its rows only).  The tail's dW GEMMs run on the side stream beside that all-gather and the
  source pass.

Loss (both forms): the truth in background + support form (``graph.SupportForm``, cont2dist's
target: background 1 off the contact set), so the O(N^2) pass streams no truth: rank p takes the
bulk over its tile range and the support rows of its block (``hicgat_pairdist_mse_fused_support_range``),
and the fp64 all-reduce sums the partial moments and dcoords.  A truth without a support form
falls back to the dense band of the rank's tile range.

Strong scaling: the step is the same whole-graph step as on one GPU; results equal the 1-GPU step
up to the summation order of the partial sums (tests/test_dist_gloo.py, world 1 / 2 / 3).

The trainer talks to a kernel object (``hicgat.kernels.HipKernels`` in production) and a comm
object (``DistComm`` over torch.distributed; ``SimComm`` runs ONE rank's share with the collectives
left out, for the per-rank compute measurement of bench.py --simulate-world), so the partitioning
and collectives are testable on CPU with gloo and a torch stand-in.
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from . import ops, streams
from .ops import _ACTS, weight_grad
from .optim import FlatAdam

TILE = 128
MODES = ("slab", "xagg", "allgather")
# "auto" (bench.py's default): the form measured faster per world size on the N = 20000 graph
# (bench.py --simulate-world).  Round 3 (profiles/r03*_simrank_*): slab at P = 2 (1.37 vs 1.48 ms
# modeled: 10000-row shards kept its replicated lin_l GEMMs cheap next to the xagg edge pass), xagg
# from P = 4 (P = 8: 0.71 vs 0.84 ms).  Round 5, with the packed one-kernel tail and the emulated
# collectives: xagg at P = 2 too (1.234 vs 1.279 ms, profiles/r05af_simrank_xagg_P2.json,
# r05y_simrank_auto_P2.json)
AUTO_XAGG_MIN_P = int(os.environ.get("HICGAT_AUTO_XAGG_MIN_P", "2"))


def resolve_mode(mode, P):
    if mode == "auto":
        return "xagg" if P >= AUTO_XAGG_MIN_P else "slab"
    return mode
# workgroups of the xagg step's side-stream grouped weight-gradient launch (beside the edge pass,
# which needs the CUs: the grouped launch's default 512 would crowd it).  Rank 0 of the simulated
# 8-rank step, emulated collectives, two sweeps (profiles/r05j_sim_ab.txt): 128: 0.477 / 0.475,
# 192: 0.472 / 0.474, 256: 0.473 / 0.469, 384: 0.475 / 0.477, 512: 0.479 / 0.477, 1024: 0.487 /
# 0.489 ms; the tail's gradients and bucket alone on the side stream (the heads' dW and the GATConv
# bucket after the edge pass): 0.495 / 0.497 (removed)
XAGG_SIDE_WGS = int(os.environ.get("HICGAT_XAGG_SIDE_WGS", "256"))
# that launch's bound below which a dW becomes weighted column sums (kernels.param_grads_grouped
# small_m; 0: dense3's 3-row dW as an MFMA tile)
XAGG_SMALL_M = int(os.environ.get("HICGAT_XAGG_SMALL_M", "16"))
# the xagg step's side branch (grouped dW + the flat-gradient all-reduce) on the "grad" stream beside
# the edge pass; False: the same launches in the same order on the step's own stream (the serial
# order tests/test_gpu_xagg.py compares the overlapped step against)
XAGG_SIDE_BRANCH = True
# row segments of the xagg step's g sums (the g all-reduce then moves S x 8 KB) for shards of at least
# XAGG_G_SEG_MIN_ROWS rows: P = 4 0.733 -> 0.719 ms, P = 2 1.216 -> 1.211 (the g sums 51 -> 41 us);
# at P = 8 (2 700 rows) the 16 -> 10 us of the sums went to the finish's segment adds (4.9 -> 8.0 us)
# and the g all-reduce still waited for the flat-gradient one: one sum there (profiles/r06d, r06e)
XAGG_G_SEGS = int(os.environ.get("HICGAT_XAGG_G_SEGS", "8"))
XAGG_G_SEG_MIN_ROWS = 4096


def _null():
    import contextlib
    return contextlib.nullcontext()


# side streams for the MLP tail's queued parameter-gradient launches in the sharded step
# (ops.side_flush lanes; 1 = one chain as on a single GPU)
SIDE_LANES = int(os.environ.get("HICGAT_DIST_SIDE_LANES", "3"))


def partition_rows(rowptr, P):
    """Contiguous row blocks with ~nnz/P CSR entries each: bounds [P+1], block p = rows
    [bounds[p], bounds[p+1]).  Boundary p is the row whose CSR start is nearest p*nnz/P, clamped so
    that every block keeps at least one row when N >= P (a hub row holding more than nnz/P entries
    would otherwise put two cuts on the same row)."""
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
        lo = b[p - 1] + (1 if N >= P else 0)
        hi = N - (P - p) if N >= P else N
        b[p] = min(max(r, lo), hi)
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

    def __init__(self, rowptr, col, P, support_rowptr=None):
        rp = np.asarray(rowptr, dtype=np.int64)
        self.col = np.asarray(col, dtype=np.int64)
        self.rp = rp
        self.P = P
        self.N = N = rp.shape[0] - 1
        if N < P:
            raise ValueError(f"cannot shard {N} rows over {P} ranks: every rank needs at least one row")
        self.bounds = partition_rows(rp, P)
        self.counts = np.diff(self.bounds)
        self.R = R = max(1, int(self.counts.max()))
        owner = np.repeat(np.arange(P, dtype=np.int64), self.counts)
        self.owner = owner
        self.gidx = owner * R + (np.arange(N, dtype=np.int64) - self.bounds[owner])
        self.nnz = np.array([rp[self.bounds[p + 1]] - rp[self.bounds[p]] for p in range(P)], dtype=np.int64)
        nb = (N + TILE - 1) // TILE
        self.tiles = nb * (nb + 1) // 2
        self.nb = nb
        self.sbounds = None
        if support_rowptr is not None:
            srp = np.asarray(support_rowptr, dtype=np.int64)
            self.sbounds = partition_rows(srp, P)
            self.snnz = np.array([srp[self.sbounds[p + 1]] - srp[self.sbounds[p]] for p in range(P)], dtype=np.int64)

    def rows(self, rank):
        """(global first row, global end row, first buffer row)."""
        return int(self.bounds[rank]), int(self.bounds[rank + 1]), rank * self.R

    def local_csr(self, rank):
        """"allgather" form: padded rowptr [P*R + 1] (only this rank's buffer rows have edges) and
        its columns remapped to buffer rows (int32)."""
        r0, r1, q0 = self.rows(rank)
        e0, e1 = int(self.rp[r0]), int(self.rp[r1])
        rp = np.empty(self.P * self.R + 1, dtype=np.int64)
        rp[:q0 + 1] = 0
        rp[q0:q0 + (r1 - r0) + 1] = self.rp[r0:r1 + 1] - e0
        rp[q0 + (r1 - r0):] = e1 - e0
        return rp.astype(np.int32), self.gidx[self.col[e0:e1]].astype(np.int32)

    def own_csr(self, rank):
        """"slab" form, forward: rowptr [N + 1] in global numbering in which only this rank's rows
        have entries, and their (global) columns."""
        r0, r1, _ = self.rows(rank)
        e0, e1 = int(self.rp[r0]), int(self.rp[r1])
        rp = np.empty(self.N + 1, dtype=np.int64)
        rp[:r0 + 1] = 0
        rp[r0:r1 + 1] = self.rp[r0:r1 + 1] - e0
        rp[r1:] = e1 - e0
        return rp.astype(np.int32), self.col[e0:e1].astype(np.int32)

    def slab_csr(self, rank):
        """"slab" form, backward source pass: for EVERY row r, the neighbours i of r that this rank
        owns (columns in [r0, r1)), sorted -- rowptr [N + 1], col (global).  Over the ranks the slabs
        partition the CSR's entries (the graph is symmetric: i lists r iff r lists i)."""
        r0, r1, _ = self.rows(rank)
        keep = (self.col >= r0) & (self.col < r1)
        row_of = np.repeat(np.arange(self.N, dtype=np.int64), np.diff(self.rp))
        per_row = np.bincount(row_of[keep], minlength=self.N)
        rp = np.zeros(self.N + 1, dtype=np.int64)
        np.cumsum(per_row, out=rp[1:])
        return rp.astype(np.int32), self.col[keep].astype(np.int32)

    def slab_perm(self, rank):
        """For every slab entry (row j, neighbour i) of ``slab_csr``: the index of the transposed
        edge (i, j) in ``own_csr``'s entries (the "xagg" form reads its per-edge terms through it)."""
        r0, r1, _ = self.rows(rank)
        e0, e1 = int(self.rp[r0]), int(self.rp[r1])
        N = np.int64(self.N)
        own_rows = np.repeat(np.arange(r0, r1, dtype=np.int64), np.diff(self.rp[r0:r1 + 1]))
        own_keys = own_rows * N + self.col[e0:e1]                 # sorted: the CSR is row-major sorted
        srp, scol = self.slab_csr(rank)
        srows = np.repeat(np.arange(self.N, dtype=np.int64), np.diff(srp.astype(np.int64)))
        keys = scol.astype(np.int64) * N + srows
        perm = np.searchsorted(own_keys, keys)
        if perm.size and not np.array_equal(own_keys[np.minimum(perm, own_keys.size - 1)], keys):
            raise ValueError("the CSR is not structurally symmetric: a slab entry has no transposed edge")
        return perm.astype(np.int32)

    def tile_range(self, rank):
        """This rank's contiguous share of the upper-triangle loss tiles."""
        return self.tiles * rank // self.P, self.tiles * (rank + 1) // self.P

    def support_rows(self, rank):
        """This rank's block of the truth's support rows (balanced by support entries)."""
        return int(self.sbounds[rank]), int(self.sbounds[rank + 1])

    def truth_band(self, rank):
        """(row0, row1, col0): the truth rows / first column the rank's tile range reads (dense form)."""
        t0, t1 = self.tile_range(rank)
        if t1 <= t0:
            return 0, 0, 0
        I0, I1 = tri_row(t0, self.nb), tri_row(t1 - 1, self.nb)
        return I0 * TILE, min(self.N, (I1 + 1) * TILE), I0 * TILE


# ---- the collective model (bench.py --simulate-world) --------------------------------------------
# NOT measured on this pool (one-GPU boxes): stated assumptions.  RCCL on one MI355X node: 7 xGMI
# links per GPU (~153 GB/s each); a collective costs a latency term plus its bytes over the
# bus bandwidth it sustains (ring convention).  ``bench.py --gpus N`` reports the measured time of
# every collective beside these figures (``COMM_TIMERS``), so the first multi-GPU run checks them.
RCCL_LAT_US = 12.0         # small-message latency of one RCCL collective inside a captured graph
RCCL_BUS_GBS = 300.0       # sustained bus bandwidth of an all-reduce / all-gather over 8 ranks
# CU footprint of an emulated collective: RCCL launches one workgroup per channel; 16 channels of
# 256 threads is the assumption for these (<= 2.4 MB) messages on an 8-GPU xGMI node
SIM_COMM_WGS = int(os.environ.get("HICGAT_SIM_COMM_WGS", "16"))
SIM_COMM_THREADS = 256


def coll_us(kind, nbytes, P):
    """Modeled time of one collective over P ranks: all_gather moves (P-1)/P of the buffer into each
    rank, all_reduce 2 (P-1)/P of it (ring / tree bus-bandwidth convention)."""
    f = (P - 1) / P * (2.0 if kind == "all_reduce" else 1.0)
    return RCCL_LAT_US + f * nbytes / (RCCL_BUS_GBS * 1e3)


# name -> list of (start, end) torch.cuda.Event pairs (or host seconds for CPU tensors) around every
# collective; bench.py sets it to {} for its eager per-kernel pass (None: off)
COMM_TIMERS = None
MODELED = {}    # name -> (kind, bytes) of the last call of that collective (for the report)


def _record(name, kind, t, P, fn):
    MODELED[name] = (kind, t.numel() * t.element_size(), P)
    if COMM_TIMERS is None:
        return fn()
    if t.is_cuda:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        COMM_TIMERS.setdefault(name, []).append((e0, e1))
        return out
    import time
    t0 = time.perf_counter()
    out = fn()
    COMM_TIMERS.setdefault(name, []).append(time.perf_counter() - t0)
    return out


def comm_report():
    """{name: {"calls", "avg_us", "modeled_us", "bytes", "kind"}} of the collectives timed since
    ``COMM_TIMERS`` was set (after a device sync)."""
    out = {}
    for name, rec in (COMM_TIMERS or {}).items():
        if rec and isinstance(rec[0], tuple):
            us = [a.elapsed_time(b) * 1e3 for a, b in rec]
        else:
            us = [1e6 * v for v in rec]
        kind, nbytes, P = MODELED.get(name, (None, None, None))
        out[name] = {"calls": len(us), "avg_us": float(np.mean(us)), "min_us": float(np.min(us)),
                     "kind": kind, "bytes": nbytes,
                     "modeled_us": coll_us(kind, nbytes, P) if kind else None}
    return out


class DistComm:
    """Collectives over a torch.distributed group (RCCL = backend "nccl" on ROCm, or gloo).
    ``name`` labels each call for ``COMM_TIMERS`` / ``comm_report``."""

    def __init__(self, group=None):
        self.group = group
        self.P = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"

    def all_gather_inplace(self, buf, own, name="all_gather"):
        """All-gather where this rank's input ``own`` is its own chunk of ``buf`` (RCCL in place)."""
        if self.nccl:
            fn = lambda: dist.all_gather_into_tensor(buf, own, group=self.group)   # noqa: E731
        else:
            fn = lambda: dist.all_gather(list(buf.chunk(self.P)), own.clone(), group=self.group)   # noqa: E731
        _record(name, "all_gather", buf, self.P, fn)

    def all_reduce(self, t, name="all_reduce"):
        _record(name, "all_reduce", t, self.P, lambda: dist.all_reduce(t, group=self.group))

    def all_gather_list(self, out, t):
        dist.all_gather(out, t, group=self.group)


class SimComm:
    """ONE rank of a P-rank job on one GPU (bench.py --simulate-world): the rank's kernels run
    exactly as in the real step, on its real shard; each collective is EMULATED where it would be
    issued -- ``hicgat_sim_collective`` holds ``SIM_COMM_WGS`` workgroups resident for the modeled
    time (``coll_us`` of the real buffer's bytes) on that stream -- so a captured rank step shows
    the collectives' time, their overlap with kernels on other streams and their CU footprint.
    ``emulate=False``: the collectives are left out (the round-4 model added them serially).  The
    buffers the collectives would fill keep their contents."""

    def __init__(self, P, rank, emulate=True):
        self.P, self.rank, self.nccl, self.group = P, rank, True, None
        self.emulate = emulate
        self.last = None

    def begin_step(self):
        self.last = None

    def _emulate(self, name, kind, t):
        if not self.emulate or not getattr(t, "is_cuda", False):
            MODELED[name] = (kind, t.numel() * t.element_size(), self.P)
            return

        def fn():
            # collectives of one communicator run one after another in issue order whatever stream
            # issued them (ProcessGroupNCCL queues them on the communicator's own stream): each
            # emulation waits for the previous one (an event, so no extra stream joins a capture)
            from . import _lib
            lib = _lib.lib()
            cur = torch.cuda.current_stream(t.device)
            if self.last is not None:
                streams.wait(cur, self.last)
            _lib.check(lib.hicgat_sim_collective(float(coll_us(kind, t.numel() * t.element_size(), self.P)),
                                                 SIM_COMM_WGS, SIM_COMM_THREADS, _lib.stream(t.device)),
                       "hicgat_sim_collective")
            self.last = streams.record(cur)
        _record(name, kind, t, self.P, fn)

    def all_gather_inplace(self, buf, own, name="all_gather"):
        self._emulate(name, "all_gather", buf)

    def all_reduce(self, t, name="all_reduce"):
        self._emulate(name, "all_reduce", t)


class ShardedTrainer:
    def __init__(self, model, x, adj, truth, lr=1e-3, kind="mse", group=None, kern=None, mode="auto", comm=None):
        if kern is None:
            from .kernels import default
            kern = default()
        self.comm = comm if comm is not None else DistComm(group)
        mode = resolve_mode(mode, self.comm.P)
        if mode not in MODES:
            raise ValueError(f"mode must be one of {MODES}, got {mode!r}")
        self.K = kern
        self.model = model
        self.group = group
        self.P = P = self.comm.P
        self.rank = rank = self.comm.rank
        self.kind = ops.LOSS_KINDS[kind]
        if kind == "contrastive":
            truth = truth.upper()      # the contrastive loss reads truth[triu] as given
        self.mode = mode
        dev = model.conv.lin_l.weight.device
        self.cuda = dev.type == "cuda"
        N = x.shape[0]
        self.N = N
        sf = truth.support
        if sf is None and not truth.buf.is_cuda:
            from .graph import SupportForm
            sf = SupportForm.build_host(truth, 1.0)
        self.sf = sf
        plan = ShardPlan(adj.rowptr32.cpu().numpy(), adj.col32.cpu().numpy(), P,
                         support_rowptr=None if sf is None else sf.rowptr.cpu().numpy())
        self.plan = plan
        R = plan.R
        self.R = R
        self.r0, self.r1, self.q0 = plan.rows(rank)
        self.local_rows = self.r1 - self.r0
        self.q1 = self.q0 + self.local_rows
        self.local_nnz = int(plan.nnz[rank])
        self.gidx = torch.from_numpy(plan.gidx).to(dev)
        self.gidx32 = self.gidx.to(torch.int32)
        # the loss reads the coordinates straight from the padded all-gather buffer (cmap = gidx): the
        # HIP path only
        self.direct_coords = self.cuda and sf is not None
        conv = model.conv
        self.W, self.att_l, self.att_r, self.bias = conv.lin_l.weight, conv.att_l, conv.att_r, conv.bias
        self.ns = conv.negative_slope
        self.H = conv.heads
        self.D = D = conv.heads * conv.out_channels
        f32 = dict(dtype=torch.float32, device=dev)
        self.x_loc = x[self.r0:self.r1].to(dev).contiguous().float()
        # ---- the loss share: bulk tiles [t0, t1) + support rows [s0, s1) (or the dense band) ----
        self.t0, self.t1 = plan.tile_range(rank)
        if sf is not None:
            self.s0, self.s1 = plan.support_rows(rank)
            self.tband = None
        else:
            b0, b1, c0 = plan.truth_band(rank)
            self.trow0, self.tcol0 = b0, c0
            self.tband = truth.buf[b0:b1, c0:].contiguous() if b1 > b0 else torch.zeros((1, 4), **f32)
        # ---- graph and node buffers ---------------------------------------------------------------
        self.slab_nnz = None
        if mode in ("slab", "xagg"):
            rp, cl = plan.own_csr(rank)
            self.rowptr, self.col = torch.from_numpy(rp).to(dev), torch.from_numpy(cl).to(dev)
            if mode == "slab":
                rp, cl = plan.slab_csr(rank)
                self.rowptr_s, self.col_s = torch.from_numpy(rp).to(dev), torch.from_numpy(cl).to(dev)
                self.slab_nnz = int(cl.shape[0])
            self.x = x.to(dev).contiguous().float()          # the embeddings, gathered once (constant)
            rows = N                                          # node buffers in global row order
            self.a0, self.a1 = self.r0, self.r1               # own rows in buffer numbering
        else:
            rp, cl = plan.local_csr(rank)
            self.rowptr, self.col = torch.from_numpy(rp).to(dev), torch.from_numpy(cl).to(dev)
            rows = P * R                                      # rank p's rows = the p-th R-row chunk
            self.a0, self.a1 = self.q0, self.q1
        if mode == "xagg":
            Rl, F = self.local_rows, x.shape[1]
            self.X4 = torch.zeros((2, 2, Rl, F), **f32)                     # (xa, xa2) per head, own rows
            self.Y0 = torch.zeros((Rl, D), **f32)                           # out (pre-activation + bias)
            self.O = torch.zeros((Rl, D), **f32)                            # relu(out): the tail's input
            self.dout_l = torch.zeros((Rl, D), **f32)
            self.dxa = torch.zeros((Rl, 2 * F), **f32)
            self.gpart = torch.zeros((kern.edge_acc_blocks(Rl), 2 * F), **f32)   # g_src partial rows
            self.a_src = torch.zeros((N, self.H), **f32)
            self.a_dst = torch.zeros((N, self.H), **f32)
            # [g_src | g_dst] (the edge pass's partial sums) in S row segments, one buffer: the step's
            # second all-reduce; the finish adds the segments (XAGG_G_SEGS)
            S = max(1, min(XAGG_G_SEGS, Rl)) if (self.cuda and Rl >= XAGG_G_SEG_MIN_ROWS) else 1
            self.gsd = torch.zeros(S, 2, 2 * F, **f32)
            self.g_src, self.g_dst = self.gsd[:, 0], self.gsd[:, 1]
            rows = 0                                                       # no [N, D] node buffers
        self.h = torch.zeros((rows, D), **f32)
        self.out = torch.zeros((rows, D), **f32)
        self.out2 = torch.zeros((rows, D), **f32)
        self.gbuf = torch.zeros((rows, D), **f32)
        self.act = _ACTS[getattr(model, "conv_act", None)]
        # packed rows [dout (D) | row stats (4H)] (the "allgather" form all-gathers them as one buffer)
        self.pack = torch.zeros((rows, D + 4 * self.H), **f32)
        self.dh = torch.zeros((rows, D), **f32)
        self.da_src = torch.zeros((rows, self.H), **f32)
        # row stats; rows this rank does not own stay 0 forever (the slab source pass reads row r's
        # da_dst for every r: 0 there, so only the owner adds da_dst_r * att_dst into dh_r)
        self.rs = torch.zeros((N if mode == "xagg" else rows, 4 * self.H), **f32)
        self.coords_buf = torch.zeros((P * R, 3), **f32)
        # step()'s coordinates in global row order (the loss reads the padded all-gather layout
        # through gidx; the loss's finalize launch writes this reordered copy)
        self.coords_glob = torch.zeros((N, 3), **f32)
        if isinstance(self.comm, SimComm):
            # the other ranks' coordinates, which the all-gather would bring: any spread-out values
            g = torch.Generator().manual_seed(rank)
            self.coords_buf.copy_(torch.randn((P * R, 3), generator=g))
        self.dcoords = torch.zeros((N, 3), **f32)
        # one fp64 all-reduce buffer [stats (12) | dcoords (3N)]: the support-form loss writes both
        # straight into it (the finalised entries 7..11 are recomputed after the sum)
        self.red = torch.zeros(12 + 3 * N, dtype=torch.float64, device=dev)
        self.stats = self.red[:12]
        self.dc64 = self.red[12:].view(N, 3)
        self.loss = torch.zeros((), **f32)
        self.opt = FlatAdam(model.flat_parameters(), lr=lr, kern=kern)
        # gradient buckets: the GATConv's parameters lead the flat buffer (flat_parameters order)
        conv_ids = {id(p) for p in (self.W, self.att_l, self.att_r, self.bias) if p is not None}
        ends = [o + p.numel() for p, o in zip(self.opt.params, self.opt.offsets) if id(p) in conv_ids]
        firsts = [o for p, o in zip(self.opt.params, self.opt.offsets) if id(p) not in conv_ids]
        cut = (max(ends) + 3) // 4 * 4
        self.grad_split = cut if (firsts and min(firsts) >= cut) else None
        # the device's persistent streams (hicgat.streams): every trainer of a process uses the same two
        self.comm_stream = streams.get("comm", dev) if self.cuda else None
        self.grad_stream = streams.get("grad", dev) if self.cuda else None

    def captured(self, warmup=2):
        """The step as one hipGraph (kernels + RCCL collectives, "nccl" backend only): one replay
        per step removes the ~70 host launches that would otherwise bound a small per-rank shard.
        The ``warmup`` eager steps are real training steps."""
        from .graphs import CapturedStep
        if not self.comm.nccl:
            raise RuntimeError("graph capture of the sharded step needs the nccl (RCCL) backend")
        if getattr(self.opt, "step_ctr", None) is None:
            self.opt.enable_device_step()
        return CapturedStep(self.step, warmup=warmup)

    def _own(self, buf):
        return buf[self.q0:self.q0 + self.R]

    def _loss(self, coords):
        """The loss share, one fp64 all-reduce of [moments | dcoords], the finalised loss; returns
        this rank's rows of dcoords (fp32) for the tail's backward."""
        K, N = self.K, self.N
        if self.direct_coords:      # coords = the padded all-gather buffer, read through gidx
            K.fused_loss_support_range(coords, self.sf, N, self.kind, self.t0, self.t1, self.s0, self.s1, self.stats,
                                       self.loss, self.dc64, cmap=self.gidx32)
        elif self.sf is not None:
            K.fused_loss_support_range(coords, self.sf, N, self.kind, self.t0, self.t1, self.s0, self.s1, self.stats,
                                       self.loss, self.dc64)
        else:
            K.fused_loss(coords, self.tband, N, self.kind, self.t0, self.t1, self.stats, self.loss, self.dcoords,
                         row0=self.trow0, col0=self.tcol0)
            self.dc64.copy_(self.dcoords)
        self.comm.all_reduce(self.red, name="loss_all_reduce")
        # finalize + this rank's rows of dcoords narrowed to fp32, one launch
        K.loss_finalize(N, self.kind, self.stats, self.loss, dc64=self.dc64, r0=self.r0, r1=self.r1,
                        dcoords=self.dcoords,
                        reorder=(self.coords_buf, self.gidx32, self.coords_glob) if self.direct_coords else None)
        return self.dcoords[self.r0:self.r1]

    def _tail(self, o=None, heads=None):
        """Tail forward on own rows (input ``o``, default this rank's rows of ``out``), the coords
        all-gather, the loss share and its all-reduce.  ``heads`` (``ops.TailHeads``): o's rows are
        formed by the tail kernel itself from the xagg aggregates."""
        if o is None:
            o = self.out[self.a0:self.a1]
        o = o.detach().requires_grad_(True)
        own = self.coords_buf[self.q0:self.q1]
        if self.act and self.cuda and ops.fused_tail_ok(self.model, o):
            # written into the all-gather rows
            coords_loc = ops.fused_tail(self.model, o, coords_out=own, heads=heads)
        else:
            coords_loc = self.model.post_act(o) if self.act else self.model.tail(o)
            own.copy_(coords_loc.detach())
        self.comm.all_gather_inplace(self.coords_buf, self._own(self.coords_buf), name="coords_all_gather")
        # direct: the loss reads the padded buffer through gidx (no reorder launch); the returned
        # coordinates are then in that layout (``global_coords`` reorders them)
        if self.direct_coords:
            # the loss's finalize launch reorders them into coords_glob (step()'s output)
            coords = self.coords_buf
        else:
            coords = self.coords_buf.index_select(0, self.gidx)
            self.coords_glob.copy_(coords)
        self._loss(coords)
        return o, coords_loc, coords

    def global_coords(self):
        """The last step's coordinates [N, 3] in global row order."""
        return self.coords_buf.index_select(0, self.gidx)

    def step(self):
        """One training step; returns (loss, stats, coords) with coords [N, 3] in global row order
        (the coordinates the step's loss was evaluated on).  All three are the trainer's persistent
        buffers (a captured step refreshes them in place on every replay), so the next step
        overwrites them: a caller that keeps a step's values across steps (best-dSCC tracking, a
        history) must ``clone()`` them, as ``hicgat.train.train``'s callers of ``train_step`` do."""
        if hasattr(self.comm, "begin_step"):
            self.comm.begin_step()
        if self.mode == "xagg" and self.cuda:
            self.opt._reattach()     # the gradient buffer is zeroed by the step's first launch (xagg_logits)
        else:
            self.opt.zero_grad()
        self.model.train()
        if self.mode == "slab":
            self._step_slab()
        elif self.mode == "xagg":
            self._step_xagg()       # its gradient all-reduces are part of the step's backward
        else:
            self._step_allgather()
        self.opt.step(counted=self._ctr() is not None)
        return self.loss, self.stats, self.coords_glob

    def _ctr(self):
        """The optimizer's device step count when the xagg step's first launch advances it (HIP path,
        device step enabled), else None (Adam increments it itself)."""
        return self.opt.step_ctr if (self.mode == "xagg" and self.cuda and
                                     getattr(self.opt, "step_ctr", None) is not None) else None

    def _tail_bucket(self, tail_done):   # the slab / allgather forms
        """The MLP tail's gradient bucket, all-reduced on the comm stream as soon as the side lanes'
        tail dW launches are done (``tail_done``: events recorded on those lanes), beside lin_l's dW
        GEMM.  Called INSIDE the overlapped-gradients block, before ``ops.side_join`` joins the lanes
        back: a wait on a lane's event after that join is what aborted the round-5 captures
        (``hicgat.streams`` rule 2)."""
        g, cut = self.opt.grad, self.grad_split
        if cut is None:
            return
        if self.cuda:
            cs = self.comm_stream
            if tail_done:
                for ev in tail_done:
                    streams.wait(cs, ev)
            else:                       # no side stream in use: the tail's gradients are on this one
                streams.fork(cs, torch.cuda.current_stream())
            with torch.cuda.stream(cs):
                self.comm.all_reduce(g[cut:], name="grad_all_reduce_tail_bucket")
        else:
            self.comm.all_reduce(g[cut:], name="grad_all_reduce_tail_bucket")

    def _gat_bucket(self):
        """The GATConv's gradient bucket (or the whole buffer when there is no split), then the
        optimizer's stream joins the comm stream."""
        g, cut = self.opt.grad, self.grad_split
        if cut is None:
            self.comm.all_reduce(g, name="grad_all_reduce")
            return
        self.comm.all_reduce(g[:cut], name="grad_all_reduce_gat_bucket")
        if self.cuda:
            streams.join(torch.cuda.current_stream(), self.comm_stream)

    def _side_event(self):
        """Events after the side streams' queued work (the tail's dW GEMMs), or None (CPU)."""
        return ops.side_record() if self.cuda else None

    def _step_slab(self):
        K, N, D, H = self.K, self.N, self.D, self.H
        r0, r1 = self.r0, self.r1
        W, al, ar = self.W.detach(), self.att_l.detach(), self.att_r.detach()
        bias = self.bias.detach()
        # ---- forward: h and the logits for every row (x replicated), aggregation of own rows ------
        _, a_src, a_dst = K.linear_att(self.x, W, al, ar, h=self.h)
        K.agg_fwd_act(self.rowptr, self.col, r0, r1, self.h, a_src, a_dst, bias, self.ns, self.act,
                      self.out, self.out2, self.rs)
        o, coords_loc, coords = self._tail()
        # ---- backward -----------------------------------------------------------------------
        dout = self.pack[:, :D]
        with ops.overlapped_param_grads(self.cuda and ops.OVERLAP_DEFAULT, hold_big=False):
            coords_loc.backward(self.dcoords[r0:r1])
            self.gbuf[r0:r1].copy_(o.grad)
            K.agg_bwd_rows(r0, r1, self.act, self.gbuf, self.out, bias, self.out2, dout, self.rs)
            fork = ops.side_mark()   # the tail's queued dW / db launches run beside the source pass
            if not self.act:
                dout[r0:r1].copy_(self.gbuf[r0:r1])
            # source pass over every row r, restricted to the neighbours this rank owns: partial
            # dh_r / da_src_r (complete when summed over ranks -- through dW and datt below)
            K.agg_bwd_src(self.rowptr_s, self.col_s, 0, N, self.h, a_src, a_dst, self.rs, dout, al, ar, self.ns,
                          self.dh, self.da_src, round_robin=True)
            ops.side_flush(after=fork, lanes=SIDE_LANES)
            self._tail_bucket(self._side_event())
            with torch.no_grad():
                # lin_l's partial dW over all rows (x replicated) on a side stream of its own (lane 2:
                # beside the tail's dW GEMMs on lane 0, not queued behind them), the GAT parameter
                # column sums beside it on this stream
                with ops._side(self.dh, self.x, lane=2):
                    if self.cuda:
                        weight_grad(K, self.dh, self.x, out=self.W.grad, accumulate=True)
                    else:
                        self.W.grad.addmm_(self.dh.t(), self.x)
            dbias = self.bias.grad if self.bias is not None else torch.empty(D, device=self.h.device)
            K.param_grad(self.h, None, self.da_src, None, H, out=(self.att_l.grad.view(-1), None, None),
                         accumulate=True)
            K.param_grad(self.h[r0:r1], dout[r0:r1].contiguous(), None, self.rs[r0:r1], H,
                         out=(None, self.att_r.grad.view(-1), dbias), accumulate=True)
        self._gat_bucket()

    def _step_xagg(self):
        """Aggregate-first GATConv (gat_xagg.hip): x replicated, every GEMM on own rows only."""
        K, D, H = self.K, self.D, self.H
        r0, r1, Rl = self.r0, self.r1, self.local_rows
        F = self.x.shape[1]
        C = D // H
        W, al, ar = self.W.detach(), self.att_l.detach(), self.att_r.detach()
        bias = self.bias.detach()
        # ---- forward ------------------------------------------------------------------------
        use_heads = self.act and self.cuda and ops.tail_heads_ok(self.model, self.O)
        # the head-fused tail's packed weights (W1c, W2c and lin_l's W) ride in the same first launch
        pk = ops.step_pack(self.model, self.O) if use_heads else None
        K.xagg_logits(self.x, W, al, ar, self.a_src, self.a_dst, zero=self.opt.grad if self.cuda else None,
                      step_ctr=self._ctr(), **({"pack": pk} if pk is not None else {}))
        K.xagg_fwd(self.rowptr, self.col, r0, r1, self.x, self.a_src, self.a_dst, self.ns, self.X4, self.rs)
        Y0 = self.Y0
        rs_own = self.rs[r0:r1]
        hc = [slice(hd * C, (hd + 1) * C) for hd in (0, 1)]
        if use_heads:
            # the head GEMMs (+ bias, relu) at the head of the one-kernel tail forward, and the rows
            # backward + dxa GEMMs at the end of its backward: four launches fewer per step
            heads = ops.TailHeads(self.X4, W.contiguous(), bias, Y0, self.dout_l, rs_own, self.dxa, act=self.act)
            with ops.prepacked(self.model, pk):
                o, coords_loc, coords = self._tail(self.O, heads=heads)
        else:
            heads = None
            # out (head hd columns) = xa^hd W_hd^T + b^hd (and relu(out) for the tail): both heads in one
            # grouped launch + one slab sum with the bias / relu epilogue; the forward needs no out2
            # (da_dst comes from dxa . xa2)
            K.gemm_rows_grouped([(self.X4[hd, 0], W[hc[hd]], Y0[:, hc[hd]], bias[hc[hd]],
                                  self.O[:, hc[hd]] if self.act else None) for hd in (0, 1)], b_kmajor=0,
                                name="gemm_fwd")
            o, coords_loc, coords = self._tail(self.O if self.act else Y0)
        # ---- backward -----------------------------------------------------------------------
        # The tail's parameter gradients (dW / db / LayerNorm sums, collected from its backward) and
        # the heads' dW_h += dout^h^T xa^h with dbias^h need only the tail's backward: ONE grouped
        # weight-gradient launch + ONE grouped column-sum launch for all of them on a side stream, then
        # the all-reduce of the whole flat gradient buffer -- both beside the edge pass.  The edge pass
        # leaves only g_src / g_dst (the attention terms' partial sums, [2, 1024]): a small grouped
        # launch, their all-reduce, and the finish that turns the SUMMED g into datt and W's att (x) g
        # term on every rank (linear in g: the same as finishing per rank and summing).  Round 4 ran
        # every gradient in one grouped launch after the edge pass and both buckets' all-reduces after
        # it (profiles/r04z3_simprof_xagg_P8_rank0_timeline.txt).
        with ops.grouped_param_grads():
            coords_loc.backward(self.dcoords[r0:r1])
        with torch.no_grad():
            if heads is None:
                K.xagg_rows_bwd(self.act, o.grad, Y0, bias, self.dout_l, rs_own)
                # dxa^hd = dout^hd W_hd, both heads in one grouped launch
                K.gemm_rows_grouped([(self.dout_l[:, hc[hd]], W[hc[hd]], self.dxa[:, hd * F:(hd + 1) * F], None,
                                      None) for hd in (0, 1)], b_kmajor=1, name="gemm_dx")
            heads = [("w", self.dout_l[:, hd * C:(hd + 1) * C], self.X4[hd, 0], self.W.grad[hd * C:(hd + 1) * C],
                      None if self.bias is None else self.bias.grad[hd * C:(hd + 1) * C]) for hd in (0, 1)]
            side = None
            if self.cuda and XAGG_SIDE_BRANCH:
                side = self.grad_stream
                streams.fork(side, torch.cuda.current_stream())
            # g_src = column sums of the edge pass's partial rows, g_dst^h = sum_i da_dst_i^h x_i over own
            # rows: tall sums (rows / 2 and rows), taken in the S row segments of gsd -- S x the blocks of
            # one sum per column chunk (profiles/r06b: 51 us at P = 2, 16 at P = 8 as one sum)
            if self.cuda:
                g_jobs = [("c", self.gpart, self.g_src, False)] + [
                    ("c", self.x[r0:r1], self.g_dst[:, hd * F:(hd + 1) * F], False, rs_own[:, 3 * H + hd])
                    for hd in range(H)]
            else:
                g_jobs = [("c", self.gpart, self.g_src[0], False),
                          ("w", rs_own[:, 3 * H:4 * H], self.x[r0:r1], self.g_dst[0].view(H, F), None, False)]
            # (the side work captured after the edge pass instead -- the edge pass first in the graph's
            # order -- measured slower: 0.485 / 0.491 vs 0.468 / 0.470 ms, profiles/r05l_sim_ab.txt)
            # Buffers on the two branches until the join below.  The side branch reads dout_l, X4[:, 0],
            # rs_own's columns, the tail's saved tensors, and reads + writes the flat gradient opt.grad
            # (every gradient but the attention vectors', which stay 0 until the finish, and W's
            # att (x) g term) through its all-reduce.  This branch (the edge pass, g's column sums and
            # all-reduce) reads x, a_src, a_dst, rs, dxa, X4[:, 1] and writes ONLY gpart and gsd --
            # nothing on it may touch opt.grad before the join (tests/test_gpu_xagg.py checks the
            # numbers with a communicator whose all-reduce really changes the buffer).
            with torch.cuda.stream(side) if side is not None else _null():
                streams.stamp("grad_begin")
                keep = ops.grouped_flush(K, heads, target_wgs=XAGG_SIDE_WGS, small_m=XAGG_SMALL_M)
                # every gradient but the attention vectors' (0 until the finish) and W's att (x) g term
                self.comm.all_reduce(self.opt.grad, name="grad_all_reduce")
                streams.stamp("grad_end")
            streams.stamp("edge_begin")
            K.xagg_edge_acc(self.rowptr, self.col, r0, r1, self.x, self.a_src, self.a_dst, self.rs, self.dxa, self.ns,
                            self.gpart, xa2=self.X4[:, 1])
            streams.stamp("edge_end")
            ops.grouped_flush(K, g_jobs)
            self.comm.all_reduce(self.gsd, name="g_all_reduce")
            if side is not None:
                streams.join(torch.cuda.current_stream(), side)
            del keep
            K.xagg_param_finish(W, al, ar, self.g_src if self.cuda else self.g_src[0],
                                self.g_dst if self.cuda else self.g_dst[0], self.W.grad, self.att_l.grad.view(-1),
                                self.att_r.grad.view(-1))

    def _step_allgather(self):
        K, D = self.K, self.D
        q0, q1 = self.q0, self.q1
        W, al, ar = self.W.detach(), self.att_l.detach(), self.att_r.detach()
        # ---- forward ------------------------------------------------------------------------
        K.linear_att(self.x_loc, W, al, ar, h=self.h[q0:q1])
        self.comm.all_gather_inplace(self.h, self._own(self.h), name="h_all_gather")
        a_src, a_dst = K.att_logits(self.h, al, ar)
        K.agg_fwd_act(self.rowptr, self.col, q0, q1, self.h, a_src, a_dst, self.bias.detach(), self.ns, self.act,
                      self.out, self.out2, self.rs)
        o, coords_loc, coords = self._tail()
        # ---- backward -----------------------------------------------------------------------
        with ops.overlapped_param_grads(self.cuda and ops.OVERLAP_DEFAULT, hold_big=False):
            coords_loc.backward(self.dcoords[self.r0:self.r1])
            dout, rs_all = self.pack[:, :D], self.pack[:, D:]
            self.gbuf[q0:q1].copy_(o.grad)
            # act: writes dout = g * relu'(out) straight into the packed rows; otherwise dout is g
            K.agg_bwd_rows(q0, q1, self.act, self.gbuf, self.out, self.bias.detach(), self.out2, dout, self.rs)
            fork = ops.side_mark()   # the tail's queued dW / db launches run beside the all-gather + source pass
            if not self.act:
                dout[q0:q1].copy_(self.gbuf[q0:q1])
            rs_all[q0:q1].copy_(self.rs[q0:q1])
            self.comm.all_gather_inplace(self.pack, self._own(self.pack), name="pack_all_gather")
            K.agg_bwd_src(self.rowptr, self.col, q0, q1, self.h, a_src, a_dst, rs_all, dout, al, ar, self.ns,
                          self.dh, self.da_src)
            ops.side_flush(after=fork, lanes=SIDE_LANES)
            self._tail_bucket(self._side_event())
            dbias = self.bias.grad if self.bias is not None else torch.empty(D, device=self.h.device)
            with torch.no_grad():
                # lin_l's dW on the side stream (joined before the gradient all-reduce), param_grad
                # beside it on this stream
                with ops._side(self.dh, self.x_loc):
                    if self.cuda:
                        weight_grad(K, self.dh[q0:q1], self.x_loc, out=self.W.grad, accumulate=True)
                    else:
                        self.W.grad.addmm_(self.dh[q0:q1].t(), self.x_loc)
            K.param_grad(self.h[q0:q1], dout[q0:q1].contiguous(), self.da_src[q0:q1], self.rs[q0:q1], self.H,
                         out=(self.att_l.grad.view(-1), self.att_r.grad.view(-1), dbias), accumulate=True)
        self._gat_bucket()

