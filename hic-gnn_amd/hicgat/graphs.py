"""hipGraph capture of a whole training step (forward, fused loss, backward, Adam).

Every kernel of the step is stream-ordered and allocation-free inside the C ABI, the tensors the
autograd functions allocate come from the graph's private pool, and ``FlatAdam`` keeps its step
count on the device (``enable_device_step``), so one captured step replays as the next step.
Replays produce the same bits as eager steps (tests/test_gpu_parity.py).

The capture runs on the device's persistent "capture" stream and its warm-up on "warm"
(``hicgat.streams``), and the streams ledger checks every fork / join of the step while it is
captured (``streams.CaptureError`` instead of an unjoined or mis-attached side stream reaching the
runtime's ``capture_end``).
"""
import torch

from . import streams


class CapturedStep:
    """``fn()`` -> outputs; captured once (after ``warmup`` eager calls on a side stream), then
    ``__call__`` replays the graph and returns the same output tensors (refreshed in place)."""

    def __init__(self, fn, warmup=2):
        cur = torch.cuda.current_stream()
        dev = cur.device
        if warmup:
            s = streams.get("warm", dev)
            streams.fork(s, cur)
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    fn()
            streams.join(cur, s)
        self.graph = torch.cuda.CUDAGraph()
        cap = streams.get("capture", dev)
        # thread_local: only this thread is in capture mode, so a concurrent thread's legal stream
        # queries (the RCCL process group's watchdog polls its work events) do not invalidate it
        err = None
        with torch.cuda.graph(self.graph, stream=cap, capture_error_mode="thread_local"):
            streams.begin_capture(cap)
            try:
                self.out = fn()
            except BaseException as exc:   # end the ledger's capture, then let torch end the graph's
                err = exc
            finally:
                try:
                    streams.end_capture()
                except streams.CaptureError as exc:
                    err = err or exc
        if err is not None:
            raise err
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
