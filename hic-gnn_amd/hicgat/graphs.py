"""hipGraph capture of a whole training step (forward, fused loss, backward, Adam).

Every kernel of the step is stream-ordered and allocation-free inside the C ABI, the tensors the
autograd functions allocate come from the graph's private pool, and ``FlatAdam`` keeps its step
count on the device (``enable_device_step``), so one captured step replays as the next step.
Replays produce the same bits as eager steps (tests/test_gpu_parity.py).
"""
import torch


class CapturedStep:
    """``fn()`` -> outputs; captured once (after ``warmup`` eager calls on a side stream), then
    ``__call__`` replays the graph and returns the same output tensors (refreshed in place)."""

    def __init__(self, fn, warmup=2):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        # thread_local: only this thread is in capture mode, so a concurrent thread's legal stream
        # queries (the RCCL process group's watchdog polls its work events) do not invalidate it
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.out = fn()
        self.fn = fn

    def __call__(self):
        self.graph.replay()
        return self.out


def captured_train_step(model, opt, x, edge_index, truth, kind="mse", warmup=2):
    """A ``CapturedStep`` of ``hicgat.train.train_step``; ``opt`` must be a ``FlatAdam``.
    The ``warmup`` eager steps are real training steps."""
    from .train import train_step
    if getattr(opt, "step_ctr", None) is None:
        opt.enable_device_step()
    stats = torch.empty(12, dtype=torch.float64, device=x.device)
    return CapturedStep(lambda: train_step(model, opt, x, edge_index, truth, kind, stats), warmup=warmup)
