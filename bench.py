"""Benchmark: GAT-HiC training steps/sec on MI355X (BASELINE.json metric).

  python bench.py [--gpus N --steps K --warmup W] [--workload synth-20000|synth-2000]

One step = zero_grad + GATConv (MFMA lin_l + fused logits, edge-softmax aggregation) + MLP tail
+ fused distance/MSE loss + backward + Adam, over the whole synthetic Hi-C graph, inputs resident
in HBM.  N > 1 (torch.distributed.run, one rank per GPU, RCCL): destination rows are sharded
across ranks with RCCL all-gathers of the 512-d node embeddings (strong scaling: the same
N = 20000 graph is split, so ``value`` = whole-model steps per second).

Rank 0 prints ONE JSON line.  ``roofline`` is computed from HIP events recorded around every
launch of the dominant kernel inside the timed region; ``cpu_baseline`` times the CPU oracle (a
plain-torch restatement of the reference path) on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "hic-gnn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); measured float4 copy ~6290
D_FEAT = 512
HEADS = 2


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def agg_bytes(kind, n, nnz, d=D_FEAT, h=HEADS):
    """Algorithmic HBM bytes per launch (DESIGN.md 'Roofline')."""
    if kind == "gat_agg_fwd":      # gather h_j + col per edge, write out + out2 (training form), rowptr, stats
        return nnz * (4 * d + 4) + 2 * n * 4 * d + (n + 1) * 4 + 2 * n * h * 4 + nnz * 4 * h + n * 16
    if kind == "gat_agg_bwd_rows":  # stream g, y, out2 in and dout out; S3 in, (delta, da_dst) out
        return 4 * n * 4 * d + 2 * n * 16
    if kind == "gat_agg_bwd_dst":  # gather h_j + col + a_src_j per edge, read dout_i
        return nnz * (4 * d + 4 + 4 * h) + n * 4 * d + (n + 1) * 4 + 5 * n * h * 4
    if kind == "gat_agg_bwd_src":  # gather dout_i + col + (a_dst, max, sum, delta)_i, read h_r, write dh_r
        return nnz * (4 * d + 4 + 16 * h) + 2 * n * 4 * d + (n + 1) * 4 + 4 * n * h * 4
    if kind == "sage_agg":          # f1 SAGEConv: gather x_j (4d) + col + weight per edge, read x_i (trunc), write z [N, 2d]
        return nnz * (4 * d + 8) + n * 4 * d + n * 8 * d + (n + 1) * 4 + n * 4
    if kind == "pairdist_mse_fused":  # upper-triangle tiles of T once + partial slabs
        nb = (n + 127) // 128
        tiles = nb * (nb + 1) // 2
        return tiles * 128 * 128 * 4 + tiles * 2 * 128 * 16 * 2
    raise KeyError(kind)


# timer name (kernels.py) -> HIP kernels launched inside that timed region
PMC_KERNELS = {
    "gat_agg_fwd": ["agg_fwd_h2c256_kernel", "agg_edge_rec_kernel", "agg_fwd_strip_kernel"],
    "gat_agg_bwd_dst": ["agg_bwd_dst_h2c256_kernel"],
    "gat_agg_bwd_rows": ["agg_bwd_rows_kernel"],
    "sage_agg": ["sage_agg_f512_kernel", "sage_agg_generic_kernel"],
    "gat_agg_bwd_src": ["agg_bwd_src_h2c256_kernel", "agg_src_rec_kernel", "agg_bwd_src_strip_kernel",
                        "agg_src_finalize_kernel"],
    "pairdist_mse_fused": ["pairdist_tile_kernel<0", "pairdist_reduce_kernel", "moments_reduce_kernel"],
}


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of ``kernel`` from the newest committed PMC summary for ``workload``
    (profiles/*pmc_traffic*.json, written by tools/pmc_traffic.py from two rocprofv3 --pmc passes
    of this bench: FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE).  None if not collected."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json"))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("workload") == workload:
            best = d
    if best is None:
        return None
    tot, seen = 0.0, False
    for pat in PMC_KERNELS[kernel]:
        for name, v in best["kernels"].items():
            if pat in name:
                tot += v["bytes"]
                seen = True
    return tot if seen else None


def build_workload(name, seed, device):
    import hicgat
    from hicgat import synth
    spec = synth.WORKLOADS[name]
    n = spec["n"]
    t0 = time.time()
    i, j, c = synth.contact_pairs(n, density=spec["density"], seed=seed)
    A = synth.dense_contacts(n, i, j, c, device=device)
    adj = hicgat.Adj.from_dense_device(A, keep_host=False)
    truth = hicgat.Truth.from_contacts(A, 0.5)
    del A
    x = torch.tensor(synth.features(n, seed=seed), device=device)
    torch.cuda.synchronize()
    log(f"[bench] workload {name}: N={n} nnz(with self loops)={adj.device_nnz} setup {time.time() - t0:.1f}s")
    return dict(n=n, pairs=(i, j, c), adj=adj, truth=truth, x=x)


def cpu_baseline(wl, seed, steps=2, warmup=1):
    """The oracle (plain-torch restatement of the reference CPU path) on the same workload."""
    from oracle import gat as og
    from oracle import graph as ogr
    from oracle import loop as ol
    from hicgat import synth
    n = wl["n"]
    i, j, c = wl["pairs"]
    rows = np.concatenate([i, j])
    cols = np.concatenate([j, i])
    order = np.lexsort((cols, rows))
    rows, cols = rows[order], cols[order]
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(rowptr, rows + 1, 1)
    adj = (torch.tensor(np.cumsum(rowptr)), torch.tensor(cols.astype(np.int64)))
    y = torch.zeros((n, n), dtype=torch.float64)
    y[torch.tensor(i), torch.tensor(j)] = torch.tensor(c)
    y[torch.tensor(j), torch.tensor(i)] = torch.tensor(c)
    truth = ogr.cont2dist(y, 0.5)
    del y
    x = torch.tensor(synth.features(n, seed=seed))
    torch.manual_seed(0)
    model = og.GATNetSelectiveResidualsUpdated()
    times = []

    def on_step(k, lv):
        times.append(time.perf_counter())
        log(f"[cpu] step {k} loss {lv:.6g}")

    t0 = time.perf_counter()
    ol.train(model, x, adj, truth, steps=warmup + steps, on_step=on_step)
    dt = times[-1] - times[warmup - 1] if warmup > 0 else times[-1] - t0
    return dict(value=steps / dt, unit="steps/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{steps} timed steps (after {warmup} warm-up) of the full {n}-node step "
                       f"(oracle GATNetSelectiveResidualsUpdated, fwd+MSE+bwd+Adam, "
                       f"{torch.get_num_threads()} threads, {os.cpu_count()} host CPUs visible)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="synth-20000", choices=["synth-20000", "synth-2000"])
    ap.add_argument("--loss", default="mse", choices=["mse", "combined"])
    ap.add_argument("--model", default="GATNetSelectiveResidualsUpdated",
                    choices=["GATNetSelectiveResidualsUpdated", "GATNetHeadsChanged3LayersLeakyReLUv2", "Net"],
                    help="the flagship (default), the v2 GAT model or the SAGE baseline Net (SURVEY 8(f) f1); "
                         "N > 1 shards the GAT models only")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python each step instead of replaying the step as one "
                         "captured hipGraph (the default; at N > 1 the graph holds the RCCL collectives too; the "
                         "per-kernel timing then comes from an eager pass of the same length right after the "
                         "timed region)")
    ap.add_argument("--graph", action="store_true", help=argparse.SUPPRESS)   # the default; kept for old scripts
    args = ap.parse_args()
    args.graph = not args.eager

    import hicgat
    from hicgat import kernels

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    wl = build_workload(args.workload, args.seed, dev)
    torch.manual_seed(0)
    model = hicgat.MODELS[args.model]().to(dev)
    if world > 1 and args.model == "Net":
        raise SystemExit("the sharded step covers the GAT models (Net is the single-GPU f1 baseline)")
    if world > 1:
        from hicgat import dist as hdist
        runner = hdist.ShardedTrainer(model, wl["x"], wl["adj"], wl["truth"], lr=1e-3, kind=args.loss)
        step = runner.step
    else:
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
        stats = torch.empty(12, dtype=torch.float64, device=dev)

        def step():
            return hicgat.train.train_step(model, opt, wl["x"], wl["adj"], wl["truth"], args.loss, stats)

    eager_step = step
    if args.graph and world > 1:
        try:
            step = runner.captured(warmup=max(1, args.warmup))   # kernels + RCCL collectives in one graph
        except RuntimeError as exc:   # keep a number on record: eager RCCL steps instead of the graph
            log(f"[bench] rank {rank}: graph capture of the sharded step failed ({exc}); timing eager steps")
            torch.cuda.synchronize()
            args.graph = False
            for w in range(args.warmup):
                step()
    elif args.graph:
        step = hicgat.graphs.captured_train_step(model, opt, wl["x"], wl["adj"], wl["truth"], args.loss,
                                                 warmup=max(1, args.warmup))
    else:
        for w in range(args.warmup):
            step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    log(f"[bench] warmup done ({args.warmup} steps)")

    if not args.graph:
        kernels.TIMERS = {}
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        loss = step()[0]
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        torch.distributed.barrier()
    if args.graph:
        kernels.TIMERS = {}
        for k in range(args.steps):
            eager_step()
        torch.cuda.synchronize()
    timers, kernels.TIMERS = kernels.TIMERS, None
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_v = float(loss.item())

    kern = {}
    for name, evs in timers.items():
        ms = [a.elapsed_time(b) for a, b in evs]
        kern[name] = dict(launches=len(ms), avg_ms=float(np.mean(ms)), total_ms=float(np.sum(ms)))
    n, nnz = wl["n"], wl["adj"].device_nnz
    if world > 1:
        nnz = runner.local_nnz
        n_loc = runner.local_rows
    else:
        n_loc = n
    cands = [k for k in ("gat_agg_fwd", "gat_agg_bwd_dst", "gat_agg_bwd_rows", "gat_agg_bwd_src", "sage_agg",
                         "pairdist_mse_fused") if k in kern]
    dom = max(cands, key=lambda k: kern[k]["total_ms"])

    def per_launch(k, b):
        """A pass split into row chunks (the source pass, ops._src_chunks) is several launches per
        step over near-equal row ranges: each launch's algorithmic bytes are the pass's share."""
        return b / max(1.0, kern[k]["launches"] / args.steps)
    if dom == "pairdist_mse_fused":
        alg = agg_bytes(dom, n, nnz) / (world if world > 1 else 1)
    else:
        alg = per_launch(dom, agg_bytes(dom, n_loc, nnz))
    achieved = alg / (kern[dom]["avg_ms"] * 1e-3) / 1e9
    for k in cands:
        b = per_launch(k, agg_bytes(k, n if k == "pairdist_mse_fused" else n_loc, nnz))
        kern[k]["alg_GBps"] = b / (kern[k]["avg_ms"] * 1e-3) / 1e9

    traffic = pmc_traffic(dom, args.workload) if world == 1 else None
    result = {
        "metric": f"training steps/sec ({args.model}, fwd+loss+bwd+Adam)",
        "value": args.steps / elapsed,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (power-law Hi-C contacts, 0.1*N(0,1) features, random-init weights seed 0)",
        "graph": bool(args.graph),
        "config": {"workload": args.workload, "model": args.model,
                   "n_nodes": n, "nnz_with_self_loops": wl["adj"].device_nnz, "d": D_FEAT, "heads": HEADS,
                   "loss": args.loss, "parallelism": f"dst-row shard x{world}" if world > 1 else "single",
                   "gemm": {0: "auto (x3 split where supported)", 1: "fp32 MFMA", 2: "x3 split"}[kernels.default().gemm_impl],
                   "aggregation": (f"xcd column strips x{kernels.default().slice_width}"
                                   if kernels.default().slice_width else "row per wave")},
        "final_loss": loss_v,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "alg_bytes_per_launch": alg, "avg_launch_ms": kern[dom]["avg_ms"],
                     "launches_per_step": kern[dom]["launches"] / args.steps,
                     # the HBM bytes the kernel really moves (PMC) over the same launch time: frac > 1
                     # above because the gathered rows are largely L2 / Infinity-Cache hits
                     "traffic_GBps": traffic / (kern[dom]["avg_ms"] * 1e-3) / 1e9 if traffic else None,
                     "traffic_frac": traffic / (kern[dom]["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS if traffic else None},
        "kernels": kern,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "GATNetSelectiveResidualsUpdated":
        log("[bench] cpu baseline (oracle) ...")
        result["cpu_baseline"] = cpu_baseline(wl, args.seed, steps=args.cpu_steps)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
