"""``FlatAdam``: torch.optim.Adam semantics (HiC-GNN_main.py:118,130) on one flat buffer.

All parameters of the model are re-pointed into one contiguous fp32 buffer and their ``.grad``
into another, so one ``hicgat_adam_step`` launch updates every parameter and a data-parallel run
all-reduces one contiguous gradient buffer (one RCCL call).  Shared parameters (GATConv's
lin_l / lin_r) are one tensor and appear once, as in ``model.parameters()``.
"""
import torch

from . import kernels


class FlatAdam:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, kern=None):
        self.kern = kern
        self.params = [p for p in params if p.requires_grad]
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        # keep every view 16-byte aligned
        offs, o = [], 0
        for p in self.params:
            offs.append(o)
            o += (p.numel() + 3) // 4 * 4
        self.numel = o
        self.flat = torch.zeros(o, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(o, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(o, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(o, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                view = self.flat[off:off + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.grad = self.grad[off:off + p.numel()].view_as(p)
                p._hicgat_grad_sink = True   # hicgat ops add their gradient straight into p.grad
        self.offsets = offs
        self.n_params = n
        self.lr, self.betas, self.eps = lr, betas, eps
        self.step_count = 0

    def enable_device_step(self, max_steps=1 << 20):
        """Keep the step count on the device so ``step()`` can be captured in a hipGraph and
        replayed.  The per-step constants are tabulated on the host with libm pow in float64 --
        the same arithmetic as the eager path (and as torch's Python-float bias corrections)."""
        import numpy as np
        lr, (b1, b2) = self.lr, self.betas
        t = np.arange(1, max_steps + 1, dtype=np.float64)
        tab = np.empty((max_steps, 2), dtype=np.float32)
        tab[:, 0] = -(lr / (1.0 - np.power(b1, t)))
        tab[:, 1] = np.power(1.0 - np.power(b2, t), 0.5)
        self.table = torch.from_numpy(tab).to(self.flat.device)
        self.step_ctr = torch.full((1,), self.step_count, dtype=torch.int64, device=self.flat.device)
        return self

    def zero_grad(self, set_to_none=False, pack=None):
        """Zero the flat gradient buffer (``set_to_none`` is ignored: the ``.grad`` views stay).  With
        the device step count on (and a GPU buffer) the zeroing launch also advances the count, and
        the next ``step()`` reads it without its own increment launch.  ``pack`` (GPU): the one-kernel
        tail's packed weights written by the same launch (``ops.step_pack``)."""
        if self.grad.is_cuda and (pack is not None or getattr(self, "step_ctr", None) is not None):
            kern = self.kern if self.kern is not None else kernels.default()
            ctr = getattr(self, "step_ctr", None)
            # a second zero_grad before the step only zeroes (the count advances once per step)
            kern.step_begin(self.grad, None if (ctr is None or getattr(self, "_counted", False)) else ctr, pack=pack)
            self._counted = ctr is not None
        else:
            self.grad.zero_()
        self._reattach()

    def _reattach(self):
        """Restore every ``p.grad`` as its flat-buffer view if something replaced it (e.g. a torch
        ``model.zero_grad()`` setting it to None), folding a foreign gradient tensor back in."""
        for p, off in zip(self.params, self.offsets):
            g = p.grad
            view = self.grad[off:off + p.numel()]
            if g is None or g.data_ptr() != view.data_ptr():
                if g is not None:
                    view.copy_(g.reshape(-1))
                else:
                    view.zero_()
                p.grad = view.view_as(p)

    @torch.no_grad()
    def step(self, counted=False):
        """``counted``: the device step count was already advanced by an earlier launch of this step
        (``kernels.xagg_logits(step_ctr=...)``), so Adam reads it without an increment launch."""
        self._reattach()
        self.step_count += 1
        counted = counted or getattr(self, "_counted", False)
        self._counted = False
        kern = self.kern if self.kern is not None else kernels.default()
        if getattr(self, "step_ctr", None) is not None:
            kern.adam_table(self.flat, self.grad, self.exp_avg, self.exp_avg_sq, self.numel, self.betas[0],
                            self.betas[1], self.eps, self.table, self.step_ctr, counted=counted)
            return
        kern.adam(self.flat, self.grad, self.exp_avg, self.exp_avg_sq, self.numel, self.lr, self.betas[0],
                  self.betas[1], self.eps, self.step_count)

    def sync_step_count(self):
        """Bring the host ``step_count`` up to the device count: replays of a captured step advance
        only ``step_ctr`` (the host count stops at the capture), so read it back once after a run."""
        if getattr(self, "step_ctr", None) is not None:
            self.step_count = int(self.step_ctr.item())
        return self.step_count

    def state_dict(self):
        return {"step": self.sync_step_count(), "exp_avg": self.exp_avg.clone(), "exp_avg_sq": self.exp_avg_sq.clone(),
                "lr": self.lr, "betas": self.betas, "eps": self.eps}
