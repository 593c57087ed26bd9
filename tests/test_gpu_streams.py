"""GPU: the step's persistent streams and the capture ledger (hicgat.streams) on captured steps.

Round 5 saw two host aborts in the sharded capture path, both in the slab form with the simulated
communicator: a segfault in ``capture_end`` (test_simulated_ranks_run_their_shares[slab-777-3]) and
a core dump after rank 4 of ``bench.py --simulate-world 8 --dist-mode slab``, whose bare rank time
had doubled just before.  The slab step waited, inside the capture, on events of side lanes that it
had already joined back into the origin (streams rule 2; DESIGN.md section 6, "Streams and
capture").  These tests rebuild the pattern that aborted and check the ledger on the device.
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _inputs(n, density=0.05, seed=3):
    for p in (os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "hic-gnn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import hicgat
    from hicgat import synth
    i, j, c = synth.contact_pairs(n, density=density, seed=seed)
    A = synth.dense_contacts(n, i, j, c, device="cuda")
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    truth = hicgat.Truth.from_contacts(A, 0.5)
    x = torch.tensor(synth.features(n, seed=seed), device="cuda")
    return hicgat, adj, truth, x


@pytest.mark.timeout(600)
def test_sim_trainers_build_capture_replay_destroy_in_one_process():
    """bench.py --simulate-world's pattern (bench.py: timed_rank): for each of four ranks of a slab-form
    4-rank job, a ShardedTrainer(SimComm) is built, captured, replayed and destroyed -- once with the
    collectives emulated and once left out, as bench.py times every rank twice -- plus an xagg one
    per rank.  Every captured run replays the same losses, bit for bit, as an eager trainer of the same
    share, and the process's stream set does not grow (one stream per name and device)."""
    hicgat, adj, truth, x = _inputs(777)
    from hicgat import streams
    seen = None
    for r in range(4):
        for mode, emu in (("slab", True), ("slab", False), ("xagg", True)):
            res = []
            for graphed in (False, True):
                torch.manual_seed(0)
                model = hicgat.GATNetSelectiveResidualsUpdated().to("cuda")
                tr = hicgat.dist.ShardedTrainer(model, x, adj, truth, lr=1e-3, mode=mode,
                                                comm=hicgat.dist.SimComm(4, r, emulate=emu))
                if graphed:
                    step = tr.captured(warmup=1)
                    losses = [None]
                    for _ in range(3):
                        losses.append(float(step()[0]))
                    del step
                else:
                    tr.opt.enable_device_step()
                    losses = [float(tr.step()[0]) for _ in range(4)]
                torch.cuda.synchronize()
                res.append((losses, tr.opt.flat.clone()))
                del tr, model
                torch.cuda.empty_cache()
            (le, pe), (lg, pg) = res
            assert le[1:] == lg[1:] and torch.equal(pe, pg), (r, mode, emu, le, lg)
            assert all(torch.isfinite(torch.tensor(le)))
            made = streams.made()
            if seen is None:
                seen = made
            assert set(made) <= set(seen) | {(0, n) for n in streams.NAMES}
            assert all(seen[k] == made[k] for k in seen), "a named stream was re-made"
    assert len(streams.made()) <= len(streams.NAMES)


def test_ledger_rejects_a_wait_on_a_joined_lane_and_the_capture_still_ends():
    """Rule 2 on the device: a captured function that joins a side stream and then waits on one of its
    earlier events raises CaptureError (before the runtime sees the wait); the capture ends cleanly
    and the next capture on the same streams replays correctly."""
    from hicgat import _lib, graphs, streams
    lib = _lib.lib()
    x = torch.zeros(4, device="cuda")
    side, cs = streams.get("side6"), streams.get("comm")

    def bad():
        cur = torch.cuda.current_stream()
        streams.fork(side, cur)
        with torch.cuda.stream(side):
            x.add_(1)
        ev = streams.record(side)
        streams.join(cur, side)
        streams.wait(cs, ev)            # rule 2
        return x

    with pytest.raises(streams.CaptureError, match="rule 2"):
        graphs.CapturedStep(bad, warmup=0)
    assert not streams.LEDGER.active

    def good():
        cur = torch.cuda.current_stream()
        streams.fork(side, cur)
        with torch.cuda.stream(side):
            x.add_(1)
            _lib.check(lib.hicgat_sim_collective(1.0, 1, 64, _lib.stream()), "hicgat_sim_collective")
        ev = streams.record(side)
        streams.wait(cs, ev)
        with torch.cuda.stream(cs):
            x.mul_(2)
        streams.join(cur, side)
        streams.join(cur, cs)
        return x

    x.zero_()
    g = graphs.CapturedStep(good, warmup=0)
    x.zero_()
    for _ in range(3):
        g()
    torch.cuda.synchronize()
    assert x.tolist() == [14.0] * 4           # ((0 + 1) * 2 + 1) * 2 + 1) * 2
