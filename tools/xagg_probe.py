"""Time the sharded xagg step's kernels one by one on a rank's real buffers (HIP events, repeated
launches): rank ``--rank`` of a simulated ``--world``-rank step on the synth-20000 workload, after
``--steps`` captured steps.  Diagnostics for the per-rank timeline (tools/gpu_run.sh simprof)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd")]

import torch  # noqa: E402


def timeit(fn, reps=20):
    """Device time per call: a 3 ms emulated-collective kernel first keeps the GPU busy while the host
    enqueues the calls, so host launch overhead (ctypes job tables) stays out of the events."""
    from hicgat import _lib
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _lib.check(_lib.lib().hicgat_sim_collective(3000.0, 16, 256, _lib.stream(torch.device("cuda", 0))), "busy")
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--grads", action="store_true", help="break the grouped parameter-gradient launches down by job")
    a = ap.parse_args()
    import bench
    import hicgat
    from hicgat import dist as hdist
    dev = torch.device("cuda", 0)
    wl = bench.build_workload("synth-20000", 0, dev)
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(dev)
    tr = hdist.ShardedTrainer(model, wl["x"], wl["adj"], wl["truth"], lr=1e-3, mode="xagg",
                              comm=hdist.SimComm(a.world, a.rank))
    rec = []
    if a.grads:   # record the grouped launch's job lists of one eager step
        K0 = tr.K
        orig = K0.param_grads_grouped

        def spy(w, c, target=None):
            rec.append((list(w), list(c), target))
            return orig(w, c, target)
        K0.param_grads_grouped = spy
        tr.opt.enable_device_step()
        tr.step()
        K0.param_grads_grouped = orig
    step = tr.captured(warmup=2)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    K = tr.K
    r0, r1 = tr.r0, tr.r1
    F, C = 512, 256
    W = tr.W.detach()
    hc = [slice(hd * C, (hd + 1) * C) for hd in (0, 1)]
    res = {}
    res["step (graph replay)"] = timeit(step)
    res["xagg_fwd"] = timeit(lambda: K.xagg_fwd(tr.rowptr, tr.col, r0, r1, tr.x, tr.a_src, tr.a_dst, tr.ns, tr.X4, tr.rs))
    rs_save = tr.rs.clone()

    def edge():
        tr.rs.copy_(rs_save)
        K.xagg_edge_acc(tr.rowptr, tr.col, r0, r1, tr.x, tr.a_src, tr.a_dst, tr.rs, tr.dxa, tr.ns, tr.gpart,
                        xa2=tr.X4[:, 1])
    res["copy rs"] = timeit(lambda: tr.rs.copy_(rs_save))
    res["xagg_edge_acc (+ rs copy)"] = timeit(edge)
    res["xagg_edge_acc no xa2"] = timeit(lambda: K.xagg_edge_acc(tr.rowptr, tr.col, r0, r1, tr.x, tr.a_src, tr.a_dst,
                                                                  tr.rs, tr.dxa, tr.ns, tr.gpart))
    dz = torch.zeros_like(tr.dxa)
    res["xagg_edge_acc dxa = 0"] = timeit(lambda: K.xagg_edge_acc(tr.rowptr, tr.col, r0, r1, tr.x, tr.a_src, tr.a_dst,
                                                                   tr.rs, dz, tr.ns, tr.gpart))
    res["dxa grouped GEMM"] = timeit(lambda: K.gemm_rows_grouped(
        [(tr.dout_l[:, hc[hd]], W[hc[hd]], tr.dxa[:, hd * F:(hd + 1) * F], None, None) for hd in (0, 1)], b_kmajor=1))
    Kp = tr.K
    for li, (w, c, tg) in enumerate(rec):   # every grouped launch pair of the step (side, then g's)
        pre = f"grads[{li}] target {tg}:"
        res[f"{pre} both launches"] = timeit(lambda: Kp.param_grads_grouped(w, c, tg))
        if w:
            res[f"{pre} weight-gradient jobs only (+ their slab sums)"] = timeit(lambda: Kp.param_grads_grouped(w, [], tg))
        if c and w:
            res[f"{pre} column-sum jobs only"] = timeit(lambda: Kp.param_grads_grouped([], c, tg))
        for k, job in enumerate(c):
            res[f"{pre} colsum job {k} {tuple(job[0].shape)}{' weighted' if len(job) > 3 else ''}"] = \
                timeit(lambda job=job: Kp.param_grads_grouped([], [job], tg))
        for k, job in enumerate(w):
            res[f"{pre} wgrad job {k} dy {tuple(job[0].shape)} x {tuple(job[1].shape)}"] = \
                timeit(lambda job=job: Kp.param_grads_grouped([job], [], tg))
    print(f"rank {a.rank} of {a.world}: rows {tr.local_rows}, nnz {tr.local_nnz}, dxa finite "
          f"{bool(torch.isfinite(tr.dxa).all())}, |dxa| max {float(tr.dxa.abs().max()):.3e}, "
          f"denormal frac {float(((tr.dxa.abs() < 1.2e-38) & (tr.dxa != 0)).float().mean()):.3e}")
    for k, v in res.items():
        print(f"{k:72s} {v:9.1f} us")


if __name__ == "__main__":
    main()
