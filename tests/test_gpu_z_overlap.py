"""GPU: the overlap the captured steps are built for, measured inside replays, AFTER the rest of the
GPU suite (this file sorts last: by then the process has made many streams and graphs, which is
when round 5 saw two streams land on one hardware queue and run in series, gpurun_out/r05m).

Each branch of a replayed step is bracketed by ``hicgat_wall_stamp`` launches (``streams.STAMPS``,
captured into the graph at the fork / join points): the device's steady wall clock at the start and
end of the branch, on every replay.  Two branches "run beside each other" when their intervals
overlap by at least half of the shorter one; run in series they overlap by ~0.

* single GPU, synth-20000 (bench.py's workload): the tail's parameter-gradient launches on the side
  lane beside the GATConv's source-side gather (ops._GATConvFn.backward / side_flush);
* the sharded xagg step (rank 0 of 8 simulated ranks, synth-20000): the side branch (grouped dW +
  the flat-gradient all-reduce, emulated) beside the edge pass (dist.ShardedTrainer._step_xagg).
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def synth20000():
    for p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import hicgat
    from hicgat import synth
    i, j, c = synth.contact_pairs(20000, density=0.01, seed=0)
    A = synth.dense_contacts(20000, i, j, c, device="cuda")
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    truth = hicgat.Truth.from_contacts(A, 0.5)
    del A
    x = torch.tensor(synth.features(20000, seed=0), device="cuda")
    return hicgat, adj, truth, x


def _replay_intervals(step, a, b, replays=6):
    """Per replay: the (begin, end) wall-clock ticks of branches ``a`` and ``b`` (stamp names)."""
    from hicgat import streams
    S = streams.SLOTS
    out = []
    for _ in range(replays):
        streams_buf = step.stamps
        streams_buf.zero_()
        step()
        torch.cuda.synchronize()
        v = streams_buf.cpu().numpy().astype(np.int64)
        out.append(((v[S[a + "_begin"]], v[S[a + "_end"]]), (v[S[b + "_begin"]], v[S[b + "_end"]])))
    return out


def _overlap(ia, ib):
    (a0, a1), (b0, b1) = ia, ib
    assert a1 > a0 > 0 and b1 > b0 > 0, (ia, ib)
    return max(0, min(a1, b1) - max(a0, b0)) / min(a1 - a0, b1 - b0)


def _captured(fn_make):
    """Capture with the stamps on (they become graph nodes), then turn them off again."""
    from hicgat import streams
    buf = torch.zeros(len(streams.SLOTS), dtype=torch.int64, device="cuda")
    streams.STAMPS = buf
    try:
        step = fn_make()
    finally:
        streams.STAMPS = None
    step.stamps = buf
    return step


def test_single_gpu_side_lane_runs_beside_the_source_gather(synth20000):
    hicgat, adj, truth, x = synth20000
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to("cuda")
    opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
    step = _captured(lambda: hicgat.graphs.captured_train_step(model, opt, x, adj, truth, warmup=1))
    iv = _replay_intervals(step, "src", "side")
    ov = [_overlap(a, b) for a, b in iv]
    us = [((a[1] - a[0]) / 100.0, (b[1] - b[0]) / 100.0) for a, b in iv]
    print("source gather / side lane (us):", us, "overlap fraction of the shorter:", [f"{v:.2f}" for v in ov])
    assert float(np.median(ov)) >= 0.5, (us, ov)


def test_xagg_side_branch_runs_beside_the_edge_pass(synth20000):
    hicgat, adj, truth, x = synth20000
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to("cuda")
    tr = hicgat.dist.ShardedTrainer(model, x, adj, truth, lr=1e-3, mode="xagg", comm=hicgat.dist.SimComm(8, 0))
    step = _captured(lambda: tr.captured(warmup=1))
    iv = _replay_intervals(step, "edge", "grad")
    ov = [_overlap(a, b) for a, b in iv]
    us = [((a[1] - a[0]) / 100.0, (b[1] - b[0]) / 100.0) for a, b in iv]
    print("edge pass / side branch (dW + flat-gradient all-reduce) (us):", us, "overlap:", [f"{v:.2f}" for v in ov])
    assert float(np.median(ov)) >= 0.5, (us, ov)
