"""Torch-CPU stand-in for ``hicgat.kernels.HipKernels`` (TEST INFRASTRUCTURE ONLY).

Implements every kernel contract of include/hicgat.h with plain torch ops on CPU tensors, so that
``hicgat.dist.ShardedTrainer``'s partitioning and collectives can run under gloo in CI.  The math
follows the oracle (PyG 1.7.2 semantics); accumulation is float64 where it is cheap, so the
sharded-vs-single comparison isolates the bookkeeping, not rounding.
"""
import numpy as np
import torch
import torch.nn.functional as F

from oracle import loop as ol

BT = 128


def _rows(rowptr, r0, r1):
    rp = rowptr.long()
    deg = rp[r0 + 1:r1 + 1] - rp[r0:r1]
    row = torch.repeat_interleave(torch.arange(r0, r1), deg)
    col_idx = torch.arange(int(rp[r0]), int(rp[r1]))
    return row, col_idx


def _scale(n, kind):
    """The per-pair gradient factor of hicgat's loss reduction (pairdist.hip loss_scale)."""
    return float(np.float32(0.1 / (n * (n - 1) / 2))) if kind == 2 else 4.0 / (n * n)


def _tri(I, J, nb):
    return I * nb - I * (I - 1) // 2 + (J - I)


def torch_tail(hicgat):
    """Give the flagship model a plain-torch tail (models.py:637-659) for CPU tensors: the product
    tail runs on the HIP GEMM / LayerNorm kernels, which need a GPU."""
    def post_act(self, x):   # after the relu, which the trainer fuses into the aggregation
        res = self.align_densea(x)
        x = F.relu(self.norm_a(self.densea(x))) + res
        res = self.align_dense1(x)
        x = F.relu(self.norm1(self.dense1(x))) + res
        x = F.relu(self.norm2(self.dense2(x)))
        return self.dense3(x)
    hicgat.GATNetSelectiveResidualsUpdated.post_act = post_act
    hicgat.GATNetSelectiveResidualsUpdated.tail = lambda self, x: post_act(self, F.relu(x))


class CpuKernels:
    def linear_att(self, x, W, att_l, att_r, h=None):
        H, C = att_l.shape[-2], att_l.shape[-1]
        hv_ = (x.double() @ W.double().t()).float()
        if h is None:
            h = hv_
        else:
            h.copy_(hv_)
        hv = h.view(-1, H, C).double()
        return h, (hv * att_l.double()).sum(-1).float(), (hv * att_r.double()).sum(-1).float()

    def att_logits(self, h, att_l, att_r):
        H, C = att_l.shape[-2], att_l.shape[-1]
        hv = h.view(-1, H, C).double()
        return (hv * att_l.double()).sum(-1).float(), (hv * att_r.double()).sum(-1).float()

    def agg_fwd(self, rowptr, col, r0, r1, h, a_src, a_dst, bias, ns, out, row_stats):
        H = a_src.shape[1]
        C = h.shape[1] // H
        row, ei = _rows(rowptr, r0, r1)
        j = col.long()[ei]
        e = F.leaky_relu(a_src[j] + a_dst[row], ns)
        n = r1 - r0
        idx = (row - r0).view(-1, 1).expand_as(e)
        m = torch.full((n, H), float("-inf")).scatter_reduce(0, idx, e, reduce="amax", include_self=True)
        u = torch.exp(e - m[row - r0])
        s = torch.zeros((n, H)).index_add(0, row - r0, u)
        al = u / (s[row - r0] + 1e-16)
        msg = h[j].view(-1, H, C).double() * al.double().unsqueeze(-1)
        agg = torch.zeros((n, H, C), dtype=torch.float64).index_add(0, row - r0, msg)
        out[r0:r1] = (agg.view(n, H * C) + bias.double()).float()
        row_stats[r0:r1, 0:H] = m
        row_stats[r0:r1, H:2 * H] = s

    def agg_fwd_act(self, rowptr, col, r0, r1, h, a_src, a_dst, bias, ns, act, out, out2, row_stats):
        self.agg_fwd(rowptr, col, r0, r1, h, a_src, a_dst, bias, ns, out, row_stats)
        if act:
            out[r0:r1] = torch.relu(out[r0:r1])
        if out2 is None:
            return
        H = a_src.shape[1]
        C = h.shape[1] // H
        row, ei = _rows(rowptr, r0, r1)
        j = col.long()[ei]
        al, lp = self._alpha(a_src, a_dst, row_stats, row, j, ns, H)
        n = r1 - r0
        msg = h[j].view(-1, H, C).double() * (al * lp).unsqueeze(-1)
        out2[r0:r1] = torch.zeros((n, H, C), dtype=torch.float64).index_add(0, row - r0, msg).view(n, H * C).float()
        row_stats[r0:r1, 2 * H:3 * H] = torch.zeros((n, H), dtype=torch.float64).index_add(
            0, row - r0, al * lp).float()

    def agg_bwd_rows(self, r0, r1, act, g, y, bias, out2, dout, row_stats):
        H = row_stats.shape[1] // 4
        n, D = r1 - r0, y.shape[1]
        d = g[r0:r1].double()
        yy = y[r0:r1].double()
        if act:
            d = torch.where(yy > 0, d, torch.zeros_like(d))
            dout[r0:r1] = d.float()
        delta = (d * (yy - bias.double())).view(n, H, D // H).sum(-1)
        p = (d * out2[r0:r1].double()).view(n, H, D // H).sum(-1)
        s3 = row_stats[r0:r1, 2 * H:3 * H].double()
        row_stats[r0:r1, 2 * H:3 * H] = delta.float()
        row_stats[r0:r1, 3 * H:4 * H] = (p - delta * s3).float()

    def _alpha(self, a_src, a_dst, row_stats, i, j, ns, H):
        e = a_src[j] + a_dst[i]
        m = row_stats[i, 0:H]
        s = row_stats[i, H:2 * H]
        al = torch.exp(F.leaky_relu(e, ns) - m) / (s + 1e-16)
        lp = torch.where(e > 0, torch.ones_like(e), torch.full_like(e, ns))
        return al.double(), lp.double()

    def agg_bwd_dst(self, rowptr, col, r0, r1, h, a_src, a_dst, dout, ns, row_stats):
        H = a_src.shape[1]
        C = h.shape[1] // H
        row, ei = _rows(rowptr, r0, r1)
        j = col.long()[ei]
        al, lp = self._alpha(a_src, a_dst, row_stats, row, j, ns, H)
        gij = (dout[row].view(-1, H, C).double() * h[j].view(-1, H, C).double()).sum(-1)
        n = r1 - r0
        s1 = torch.zeros((n, H), dtype=torch.float64).index_add(0, row - r0, al * gij)
        s2 = torch.zeros((n, H), dtype=torch.float64).index_add(0, row - r0, al * lp * gij)
        s3 = torch.zeros((n, H), dtype=torch.float64).index_add(0, row - r0, al * lp)
        row_stats[r0:r1, 2 * H:3 * H] = s1.float()
        row_stats[r0:r1, 3 * H:4 * H] = (s2 - s1 * s3).float()

    def agg_bwd_src(self, rowptr, col, r0, r1, h, a_src, a_dst, row_stats, dout, att_l, att_r, ns, dh, da_src,
                    round_robin=False):
        H = a_src.shape[1]
        C = h.shape[1] // H
        r, ei = _rows(rowptr, r0, r1)
        i = col.long()[ei]                      # neighbours of r = rows that have r as a neighbour
        al, lp = self._alpha(a_src, a_dst, row_stats, i, r, ns, H)
        gir = (dout[i].view(-1, H, C).double() * h[r].view(-1, H, C).double()).sum(-1)
        delta = row_stats[i, 2 * H:3 * H].double()
        n = r1 - r0
        dsrc = torch.zeros((n, H), dtype=torch.float64).index_add(0, r - r0, al * lp * (gir - delta))
        acc = torch.zeros((n, H, C), dtype=torch.float64).index_add(
            0, r - r0, al.unsqueeze(-1) * dout[i].view(-1, H, C).double())
        ddst = row_stats[r0:r1, 3 * H:4 * H].double()
        acc = acc + dsrc.unsqueeze(-1) * att_l.double() + ddst.unsqueeze(-1) * att_r.double()
        dh[r0:r1] = acc.view(n, H * C).float()
        da_src[r0:r1] = dsrc.float()

    def param_grad(self, h, dout, da_src, row_stats, H, out=None, accumulate=False):
        n, D = h.shape
        C = D // H
        hv = h.view(n, H, C).double()
        want = (True, True, True) if out is None else tuple(o is not None for o in out)
        datt_l = (da_src.double().unsqueeze(-1) * hv).sum(0).reshape(-1).float() if want[0] else None
        datt_r = ((row_stats[:, 3 * H:4 * H].double().unsqueeze(-1) * hv).sum(0).reshape(-1).float()
                  if want[1] else None)
        dbias = dout.double().sum(0).float() if want[2] else None
        res = (datt_l, datt_r, dbias)
        if out is None:
            return res
        for o, r in zip(out, res):
            if o is None:
                continue
            if accumulate:
                o.add_(r)
            else:
                o.copy_(r)
        return out

    # -- GEMM / column sums (hicgat_gemm_ex, hicgat_colsum): the "xagg" step runs its GEMMs here ----
    def gemm(self, a_kmajor, b_kmajor, M, N, K, A, B, C, bias=None, accumulate=False, splits=1, name="gemm",
             impl=None):
        opA = (A.t() if a_kmajor else A)[:M, :K].double()
        opB = (B if b_kmajor else B.t())[:K, :N].double()
        r = opA @ opB
        if bias is not None:
            r = r + bias.double()
        if accumulate:
            r = r + C.double()
        C.copy_(r.float())
        return C

    def gemm_rows_grouped(self, jobs, b_kmajor, splits=None, name="gemm_grouped"):
        for A, B, C, bias, Cr in jobs:
            r = A.double() @ (B.double() if b_kmajor else B.double().t())
            if bias is not None:
                r = r + bias.double()
            C.copy_(r.float())
            if Cr is not None:
                Cr.copy_(torch.relu(C))

    def colsum(self, A, out, accumulate=False):
        r = A.double().sum(0)
        out.copy_((r + out.double()).float() if accumulate else r.float())
        return out

    # -- aggregate-first GATConv (gat_xagg.hip) -------------------------------------------------------
    def xagg_logits(self, x, W, att_l, att_r, a_src, a_dst, zero=None, step_ctr=None):
        if zero is not None:
            zero.zero_()
        H, C = att_l.shape[-2], att_l.shape[-1]
        Wd = W.double().view(H, C, -1)
        vs = torch.einsum("hc,hck->hk", att_l.double().view(H, C), Wd)
        vd = torch.einsum("hc,hck->hk", att_r.double().view(H, C), Wd)
        a_src.copy_((x.double() @ vs.t()).float())
        a_dst.copy_((x.double() @ vd.t()).float())

    def xagg_fwd(self, rowptr, col, r0, r1, x, a_src, a_dst, ns, X4, row_stats):
        H = 2
        row, ei = _rows(rowptr, r0, r1)
        j = col.long()[ei]
        e = a_src[j] + a_dst[row]
        le = F.leaky_relu(e, ns)
        n = r1 - r0
        idx = (row - r0).view(-1, 1).expand_as(le)
        m = torch.full((n, H), float("-inf")).scatter_reduce(0, idx, le, reduce="amax", include_self=True)
        u = torch.exp(le - m[row - r0])
        ssum = torch.zeros((n, H)).index_add(0, row - r0, u)
        al = (u / (ssum[row - r0] + 1e-16)).double()
        lp = torch.where(e > 0, torch.ones_like(e), torch.full_like(e, ns)).double()
        xj = x[j].double()
        for hd in range(H):
            X4[hd, 0] = torch.zeros((n, x.shape[1]), dtype=torch.float64).index_add(
                0, row - r0, al[:, hd:hd + 1] * xj).float()
            X4[hd, 1] = torch.zeros((n, x.shape[1]), dtype=torch.float64).index_add(
                0, row - r0, (al * lp)[:, hd:hd + 1] * xj).float()
        row_stats[r0:r1, 0:H] = m
        row_stats[r0:r1, H:2 * H] = ssum
        row_stats[r0:r1, 2 * H:3 * H] = torch.zeros((n, H), dtype=torch.float64).index_add(
            0, row - r0, al * lp).float()

    def xagg_bias_relu(self, y0, bias, o):
        y0.add_(bias)
        o.copy_(torch.relu(y0))

    def xagg_rows_bwd(self, act, g, y0, bias, dout, row_stats):
        H = 2
        rows, D = y0.shape
        d = g.double()
        y = y0.double()
        if act:
            d = torch.where(y > 0, d, torch.zeros_like(d))
        dout.copy_(d.float())
        delta = (d * (y - bias.double())).view(rows, H, D // H).sum(-1)
        s3 = row_stats[:, 2 * H:3 * H].clone()
        row_stats[:, 2 * H:3 * H] = delta.float()
        row_stats[:, 3 * H:4 * H] = s3

    def xagg_edge(self, rowptr, col, r0, r1, x, a_src, a_dst, row_stats, dxa, ns, ds, xa2=None):
        H = 2
        Fd = x.shape[1]
        row, ei = _rows(rowptr, r0, r1)
        j = col.long()[ei]
        al, lp = self._alpha(a_src, a_dst, row_stats, row, j, ns, H)
        g = (dxa[row - r0].double().view(-1, H, Fd) * x[j].double().unsqueeze(1)).sum(-1)
        delta = row_stats[row, 2 * H:3 * H].double()
        ds[ei - int(rowptr[r0])] = (al * lp * (g - delta)).float()
        if xa2 is not None:
            dx = dxa.double().view(r1 - r0, H, Fd)
            q = torch.stack([(dx[:, hd] * xa2[hd].double()).sum(-1) for hd in range(H)], 1)
            s3 = row_stats[r0:r1, 3 * H:4 * H].double()
            row_stats[r0:r1, 3 * H:4 * H] = (q - row_stats[r0:r1, 2 * H:3 * H].double() * s3).float()

    def edge_acc_blocks(self, rows):
        return 4

    def xagg_edge_acc(self, rowptr, col, r0, r1, x, a_src, a_dst, row_stats, dxa, ns, gpart, xa2=None):
        """hicgat_xagg_edge_acc: g_src = sum over the own rows' edges of ds_ij x_j, as partial rows
        (here all of it in row 0), and da_dst with xa2."""
        H = 2
        Fd = x.shape[1]
        row, ei = _rows(rowptr, r0, r1)
        j = col.long()[ei]
        al, lp = self._alpha(a_src, a_dst, row_stats, row, j, ns, H)
        g = (dxa[row - r0].double().view(-1, H, Fd) * x[j].double().unsqueeze(1)).sum(-1)
        ds = al * lp * (g - row_stats[row, 2 * H:3 * H].double())
        gpart.zero_()
        gpart[0] = (ds.t() @ x[j].double()).reshape(-1).float()
        if xa2 is not None:
            dx = dxa.double().view(r1 - r0, H, Fd)
            q = torch.stack([(dx[:, hd] * xa2[hd].double()).sum(-1) for hd in range(H)], 1)
            s3 = row_stats[r0:r1, 3 * H:4 * H].double()
            row_stats[r0:r1, 3 * H:4 * H] = (q - row_stats[r0:r1, 2 * H:3 * H].double() * s3).float()

    def param_grads_grouped(self, wjobs, cjobs, target_wgs=None, small_m=None):
        for dy, x, dw, db, acc in wjobs:
            r = dy.double().t() @ x.double()
            dw.copy_((r + dw.double()).float() if acc else r.float())
            if db is not None:
                b = dy.double().sum(0)
                db.copy_((b + db.double()).float() if acc else b.float())
        for src, dst, acc in cjobs:
            self.colsum(src, dst, accumulate=acc)

    def xagg_slab_sum(self, rowptr_s, perm, ds, x, da_src, g_src):
        N = da_src.shape[0]
        j, k = _rows(rowptr_s, 0, N)
        da = torch.zeros((N, 2), dtype=torch.float64).index_add(0, j, ds[perm.long()[k]].double())
        da_src.copy_(da.float())
        g_src.copy_((da.t() @ x.double()).reshape(-1).float())

    def xagg_param_finish(self, W, att_l, att_r, g_src, g_dst, dW, datt_l, datt_r):
        H, C = att_l.shape[-2], att_l.shape[-1]
        gs, gd = g_src.double().view(H, -1), g_dst.double().view(H, -1)
        al, ar = att_l.double().view(H, C), att_r.double().view(H, C)
        Wd = W.double().view(H, C, -1)
        dW.copy_((dW.double().view(H, C, -1) + al.unsqueeze(-1) * gs.unsqueeze(1)
                  + ar.unsqueeze(-1) * gd.unsqueeze(1)).view_as(dW).float())
        datt_l.copy_((datt_l.double().view(H, C) + torch.einsum("hck,hk->hc", Wd, gs)).view_as(datt_l).float())
        datt_r.copy_((datt_r.double().view(H, C) + torch.einsum("hck,hk->hc", Wd, gd)).view_as(datt_r).float())

    def num_tiles(self, n):
        nb = (n + BT - 1) // BT
        return nb * (nb + 1) // 2

    def fused_loss(self, coords, tbuf, n, kind, t0, t1, stats, loss, dcoords, row0=0, col0=0):
        """``tbuf`` = the truth or a band of it from (row0, col0) (kernels.HipKernels.fused_loss)."""
        nb = (n + BT - 1) // BT
        Tb = tbuf.double()
        c = coords.double()
        iu = torch.triu_indices(n, n, 1)
        ii, jj = iu[0], iu[1]
        tid = _tri(ii // BT, jj // BT, nb)
        keep = (tid >= t0) & (tid < t1)
        ii, jj = ii[keep], jj[keep]
        diff = c[ii] - c[jj]
        d = diff.norm(dim=1)
        t = Tb[ii - row0, jj - col0]
        r = d - t
        stats[0] = r.abs().sum() if kind == 2 else (r * r).sum()
        stats[1] = d.sum()
        stats[2] = (d * d).sum()
        stats[3] = (d * t).sum()
        stats[4] = t.sum()
        stats[5] = (t * t).sum()
        dii = torch.arange(n)
        dtile = _tri(dii // BT, dii // BT, nb)
        dkeep = (dtile >= t0) & (dtile < t1)
        stats[6] = (Tb[dii[dkeep] - row0, dii[dkeep] - col0] ** 2).sum() if kind != 2 else 0.0
        w = torch.where(d > 0, (torch.sign(r) if kind == 2 else r) / d, torch.zeros_like(d)) * _scale(n, kind)
        g = torch.zeros((n, 3), dtype=torch.float64)
        g.index_add_(0, ii, w.unsqueeze(1) * diff)
        g.index_add_(0, jj, -w.unsqueeze(1) * diff)
        dcoords.copy_(g.float())
        self.loss_finalize(n, kind, stats, loss)

    def fused_loss_support_range(self, coords, sf, n, kind, t0, t1, s0, s1, stats, loss, dcoords):
        """hicgat_pairdist_mse_fused_support_range: the bulk (every pair of the tile range at the
        background value) + the support rows [s0, s1) (their differing entries and diagonal)."""
        nb = (n + BT - 1) // BT
        c = coords.double()
        bg = float(sf.background)
        iu = torch.triu_indices(n, n, 1)
        ii, jj = iu[0], iu[1]
        tid = _tri(ii // BT, jj // BT, nb)
        keep = (tid >= t0) & (tid < t1)
        ii, jj = ii[keep], jj[keep]
        diff = c[ii] - c[jj]
        d = diff.norm(dim=1)
        r = d - bg
        m = torch.zeros(7, dtype=torch.float64)
        m[0] = r.abs().sum() if kind == 2 else (r * r).sum()
        m[1] = d.sum()
        m[2] = (d * d).sum()
        m[3] = (d * bg).sum()
        m[4] = bg * d.numel()
        m[5] = bg * bg * d.numel()
        g = torch.zeros((n, 3), dtype=torch.float64)
        w = torch.where(d > 0, (torch.sign(r) if kind == 2 else r) / d, torch.zeros_like(d))
        g.index_add_(0, ii, w.unsqueeze(1) * diff)
        g.index_add_(0, jj, -w.unsqueeze(1) * diff)
        rp = sf.rowptr.long()
        si, ei = _rows(rp, s0, s1)
        sj = sf.col_buf.long()[ei]
        t = sf.val_buf.double()[ei]
        sdiff = c[si] - c[sj]
        sd = sdiff.norm(dim=1)
        sw = torch.sign(sd - t) - torch.sign(sd - bg) if kind == 2 else bg - t
        g.index_add_(0, si, torch.where(sd > 0, sw / sd, torch.zeros_like(sd)).unsqueeze(1) * sdiff)
        up = sj > si
        su, tu = sd[up], t[up]
        if kind == 2:
            m[0] += ((su - tu).abs() - (su - bg).abs()).sum()
        else:
            m[0] += ((su - tu) ** 2 - (su - bg) ** 2).sum()
        m[3] += (su * (tu - bg)).sum()
        m[4] += (tu - bg).sum()
        m[5] += (tu * tu - bg * bg).sum()
        m[6] = (sf.diag.double()[s0:s1] ** 2).sum() if kind != 2 else 0.0
        stats[:7] = m
        gf = (g * _scale(n, kind)).float()
        dcoords.copy_(gf.to(dcoords.dtype).view_as(dcoords))
        self.loss_finalize(n, kind, stats, loss)

    def loss_finalize(self, n, kind, stats, loss, dc64=None, r0=0, r1=0, dcoords=None, reorder=None):
        if dc64 is not None:
            dcoords[r0:r1].copy_(dc64[r0:r1])
        if reorder is not None:
            cbuf, gidx, cglob = reorder
            cglob.copy_(cbuf.index_select(0, gidx.long()))
        s = stats.double()
        M = n * (n - 1) / 2
        if kind == 2:        # contrastive: 0.1 * mean_{i<j} |t - d| (fp64)
            mae = float(s[0]) / M
            stats[7], stats[8], stats[9], stats[10] = mae, float("nan"), 0.1, 0.1 * mae
            loss.fill_(0.1 * mae)
            return
        mse = (2 * float(s[0]) + float(s[6])) / (n * n)
        cov = float(s[3]) - float(s[1]) * float(s[4]) / M
        vd = float(s[2]) - float(s[1]) ** 2 / M
        vt = float(s[5]) - float(s[4]) ** 2 / M
        r = cov / np.sqrt(vd * vt) if vd > 0 and vt > 0 else float("nan")
        msef = float(np.float32(mse))
        alpha = min(1.0, 0.1 + 1.0 / (msef + 1e-6))
        total = float(np.float32(msef) + np.float32(alpha * (1 - r)))
        stats[7], stats[8], stats[9], stats[10] = mse, r, alpha, total
        loss.fill_(total if kind == 1 else msef)

    def adam(self, flat, grad, m, v, n, lr, b1, b2, eps, step):
        p2, m2, v2 = ol.adam_reference_step(flat.numpy(), grad.numpy(), m.numpy(), v.numpy(), step, lr, b1, b2, eps)
        flat.copy_(torch.from_numpy(p2))
        m.copy_(torch.from_numpy(m2))
        v.copy_(torch.from_numpy(v2))
