"""Benchmark: GAT-HiC training steps/sec on MI355X (BASELINE.json metric).

  python bench.py [--gpus N --steps K --warmup W] [--workload synth-20000|synth-2000]
                  [--dist-mode slab|allgather] [--simulate-world P]

One step = zero_grad + GATConv (MFMA lin_l + fused logits, edge-softmax aggregation) + MLP tail
+ fused distance/MSE loss + backward + Adam, over the whole synthetic Hi-C graph, inputs resident
in HBM, replayed as one captured hipGraph (``--eager``: kernel by kernel).  The W warm-up steps are
real training steps: W - 1 eager ones before the capture and the graph's first replay (which also
uploads the graph), then the K timed replays.

N > 1: one rank per GPU over RCCL (hicgat.dist: destination rows sharded by an nnz prefix sum;
"slab" form by default -- the 512-d embeddings gathered once, h recomputed per rank, the source
pass split by destination owner, so no per-step collective above the 2.4 MB gradient buffer;
``--dist-mode allgather``: the RCCL all-gather of h before the layer; strong scaling -- the same
N = 20000 graph is split, so ``value`` = whole-model steps per second).

``--simulate-world P`` (one GPU): runs each of the P ranks' shares of the sharded step in turn
with the collectives left out (hicgat.dist.SimComm), graph-captured, and reports the per-rank
step times (``simulated.rank_ms``) plus a step-time model = max over ranks + the modeled time of
the collectives that are not overlapped (``simulated``; the xGMI / RCCL figures are stated
assumptions, not measurements).  ``value`` is then that MODEL's steps/s and ``n_gpus`` is 1.  Launched by the driver through
``torch.distributed.run`` (RANK / WORLD_SIZE in the environment), or directly as
``python bench.py --gpus N``: then this script starts ``torch.distributed.run`` itself as a child
process (before any GPU call) and exits with its code; it exits non-zero if fewer than N GPUs are
visible.

Rank 0 prints ONE JSON line.  ``value`` = K / (max over ranks of the barrier-bracketed wall time of
the K timed steps).  Per-kernel times (``kernels``, ``roofline.avg_launch_ms``) come from HIP
events around every launch in an EAGER pass of K steps run right after the timed region (a graph
replay hides kernel boundaries); rocprofv3's per-kernel averages of the same command are committed
under profiles/ to cross-check them.  ``roofline.frac`` = HBM bytes the dominant kernel really
moves (PMC FETCH_SIZE x 2 + WRITE_SIZE, rocprofv3 --pmc passes recorded in profiles/*pmc_traffic*,
command and commit named in ``traffic_source``) / its average launch time / 8 TB/s;
``l2_frac`` = its SURVEY 8(d) no-reuse algorithmic bytes / time / the 34.5 TB/s L2 peak (the
gathered rows are L2 / Infinity-Cache hits).  ``cpu_baseline`` times the CPU
oracle (a plain-torch restatement of the reference path) on the same workload.

``--selftest-cpu`` (tests only): gloo ranks on the CPU with the torch stand-in kernels of
tests/cpu_kernels.py on a 400-node graph -- exercises the launcher and the sharded step; it is
not a measurement.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "hic-gnn_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); measured float4 copy ~6290
L2_PEAK_GBS = 34500.0   # MI355X aggregate L2 (MI355X_MICROARCH.md "L2 (per XCD)")
MALL_GATHER_GBS = 8600.0  # Infinity-Cache random-row gather rate, 33.5 GB/s per CU (MI355X_MICROARCH.md)
MFMA_F32_TFS = 157.3    # dense fp32 MFMA peak, v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md)
D_FEAT = 512
HEADS = 2


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def agg_bytes(kind, n, nnz, d=D_FEAT, h=HEADS):
    """Algorithmic (no-reuse) bytes per launch."""
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
    "gat_agg_fwd": ["agg_fwd_h2c256_kernel"],
    "gat_agg_bwd_dst": ["agg_bwd_dst_h2c256_kernel"],
    "gat_agg_bwd_rows": ["agg_bwd_rows_kernel"],
    "sage_agg": ["sage_agg_f512_kernel", "sage_agg_generic_kernel"],
    "gat_agg_bwd_src": ["agg_bwd_src_h2c256_kernel"],
    "pairdist_mse_fused": ["pairdist_tile_kernel<0", "pairdist_persist_kernel", "pairdist_reduce_kernel",
                           "moments_partial_kernel", "moments_final_kernel"],
}


def kernel_src_hash():
    """sha1 of the kernel sources (hic-gnn_amd/csrc/*): a PMC summary recorded with other kernel
    sources describes other kernels (tools/pmc_traffic.py and tools/pmc_mfma.py store it)."""
    import glob
    import hashlib
    h = hashlib.sha1()
    for f in sorted(glob.glob(os.path.join(ROOT, "hic-gnn_amd", "csrc", "*"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _pmc_doc(pattern, workload):
    """The newest committed PMC summary for ``workload`` recorded with the CURRENT kernel sources,
    else the newest one flagged stale: (doc, source dict) or (None, None)."""
    import glob
    cur = kernel_src_hash()
    docs = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pattern))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("workload") == workload:
            docs.append((d, f))
    if not docs:
        return None, None
    fresh = [x for x in docs if x[0].get("src_hash") == cur]
    d, f = (fresh or docs)[-1]
    return d, {"file": os.path.relpath(f, ROOT), "command": d.get("command"), "commit": d.get("commit"),
               "src_hash": d.get("src_hash"), "current_src_hash": cur, "stale": not fresh}


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of ``kernel`` from the newest committed PMC summary for ``workload``
    (profiles/*pmc_traffic*.json, written by tools/pmc_traffic.py from two rocprofv3 --pmc passes
    of this bench: FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE).  (bytes, source) or (None, None)."""
    best, src = _pmc_doc("*pmc_traffic*.json", workload)
    if best is None:
        return None, None
    tot, seen = 0.0, False
    for pat in PMC_KERNELS[kernel]:
        for name, v in best["kernels"].items():
            if pat in name:
                tot += v["bytes"]
                seen = True
    if not seen:
        return None, None
    return tot, src


def gemm_block(workload, kern_t):
    """MFMA utilisation of the GEMMs (north star: "MFMA utilisation against CDNA4 peak"): per kernel
    shape (template + grid) from the committed rocprofv3 PMC pass (profiles/*pmc_mfma*.json,
    tools/pmc_mfma.py: FLOP = SQ_INSTS_VALU_MFMA_MOPS_F32 x 512, busy = SQ_VALU_MFMA_BUSY_CYCLES /
    (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)), plus the live HIP-event time per step of each GEMM family."""
    doc, src = _pmc_doc("*pmc_mfma*.json", workload)
    out = {"peak_tflops": MFMA_F32_TFS, "source": src, "shapes": {}}
    if doc is not None:
        tot_f = tot_t = 0.0
        for k, v in doc["kernels"].items():
            if v["flop"] < 1e9:
                continue
            out["shapes"][k] = {"gflop": v["flop"] / 1e9, "tflops": v["tflops_pmc"], "frac": v["tflops_pmc"] / MFMA_F32_TFS,
                                "mfma_busy": v["mfma_busy"], "clock_ghz": v["clock_ghz"]}
            tot_f += v["flop"] * v["dispatches"]
            tot_t += v["duration_s"] * v["dispatches"]
        if tot_t > 0:
            out["weighted_tflops"] = tot_f / tot_t / 1e12
            out["weighted_frac"] = out["weighted_tflops"] / MFMA_F32_TFS
    out["live_ms_per_step"] = {k: v["total_ms"] / max(1, v["launches"]) * v["launches"] for k, v in kern_t.items()
                               if k.startswith("gemm") or k == "gat_linear_att"}
    return out


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


def build_selftest_workload(seed, n=400):
    """A small CPU workload for --selftest-cpu (no GPU, no oracle: T is any symmetric target)."""
    import hicgat
    from hicgat import synth
    i, j, c = synth.contact_pairs(n, density=0.05, seed=seed)
    adj = hicgat.Adj(torch.tensor(i), torch.tensor(j), None, (n, n)).to_symmetric().to("cpu")
    A = np.zeros((n, n))
    A[i, j] = c
    A[j, i] = c
    with np.errstate(divide="ignore"):
        t = np.where(A > 0, A ** -0.5, 0.0)
    t[A == 0] = t.max()
    np.fill_diagonal(t, 0.0)
    truth = hicgat.Truth(torch.tensor(t / t.max(), dtype=torch.float32))
    x = torch.tensor(synth.features(n, seed=seed))
    return dict(n=n, pairs=(i, j, c), adj=adj, truth=truth, x=x)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(wl, seed, steps=5, warmup=2):
    """The oracle (plain-torch restatement of the reference CPU path) on the same workload:
    ``steps`` timed steps after ``warmup``, median step time (SURVEY 8(d) 'CPU baseline')."""
    from oracle import gat as og
    from oracle import graph as ogr
    from oracle import loop as ol
    from hicgat import synth
    # the box's CPU share: OMP_NUM_THREADS (16 per GPU on the pool) or the affinity mask
    threads = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    torch.set_num_threads(threads)
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
    # parity (outside the timed CPU steps): the step-1 forward of the same seed-0 weights -- the
    # coordinates (get_model; the flagship has no dropout, so the training forward's are the same)
    # and the MSE with exact-formula distances, as the device computes them
    t_par = time.perf_counter()
    with torch.no_grad():
        c1 = model.get_model(x, adj)
        mode, og.CDIST_MODE = og.CDIST_MODE, "donot_use_mm_for_euclid_dist"
        try:
            l1_exact = float(torch.nn.functional.mse_loss(
                torch.cdist(c1, c1, p=2, compute_mode=og.CDIST_MODE).float(), truth.float()))
        finally:
            og.CDIST_MODE = mode
    log(f"[cpu] step-1 forward for parity: loss (exact cdist) {l1_exact:.9g} ({time.perf_counter() - t_par:.1f} s)")
    marks = [time.perf_counter()]

    def on_step(k, lv):
        marks.append(time.perf_counter())
        log(f"[cpu] step {k} loss {lv:.6g} ({marks[-1] - marks[-2]:.2f} s)")

    hist = ol.train(model, x, adj, truth, steps=warmup + steps, on_step=on_step)
    per = np.diff(marks)[warmup:]
    med = float(np.median(per))
    return dict(value=1.0 / med, unit="steps/s", cores=threads, kind="port",
                step1={"coords": c1.detach(), "loss_exact_cdist": l1_exact, "loss_reference_cdist": hist[0]},
                median_s_per_step=med, step_s=[float(v) for v in per], cpu_model=_cpu_model(),
                host_cpus_visible=os.cpu_count(),
                sample=f"median of {steps} timed steps (after {warmup} warm-up) of the full {n}-node step "
                       f"(oracle GATNetSelectiveResidualsUpdated, fwd+MSE+bwd+Adam, torch CPU, "
                       f"{threads} threads = the box's CPU share (OMP_NUM_THREADS), {os.cpu_count()} host CPUs "
                       f"visible, {_cpu_model()})")


PARITY_TOL = 1e-5   # BASELINE.json north star: "predicted coordinates and loss within 1e-5 relative fp32"


def parity_block(dev, cpu):
    """The device's training step 1 against the CPU oracle's step 1 on the same workload and seed-0
    weights (HiC-GNN_main.py:126-130): the loss relative to the oracle's (exact-formula distances,
    as the device computes them; the reference's mm-formula cdist value beside it)
    and the coordinates as max |difference| / max |oracle coordinate|."""
    c_dev = dev["coords"].double().cpu()
    c_cpu = cpu["coords"].double()
    coords_rel = float((c_dev - c_cpu).abs().max() / c_cpu.abs().max())
    l_ref = cpu["loss_exact_cdist"]
    loss_rel = abs(dev["loss"] - l_ref) / abs(l_ref)
    l_mm = cpu["loss_reference_cdist"]
    return {"step": 1, "loss_device": dev["loss"], "loss_oracle": l_ref, "loss_rel": loss_rel,
            "coords_rel": coords_rel, "tol": PARITY_TOL, "pass": bool(loss_rel <= PARITY_TOL and coords_rel <= PARITY_TOL),
            "loss_oracle_reference_cdist": l_mm, "loss_rel_reference_cdist": abs(dev["loss"] - l_mm) / abs(l_mm),
            "note": "device step 1 (the first eager warm-up step, seed-0 weights) vs the CPU oracle's step 1 on "
                    "the same workload: loss vs the oracle's MSE with exact-formula distances (the device's "
                    "distances); loss_oracle_reference_cdist is the oracle's own training-loop value with torch's "
                    "mm-formula cdist (the reference's arithmetic, SURVEY fact 8)"}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args):
    """``python bench.py --gpus N`` without a torch.distributed.run environment: start one as a
    child process (no GPU call has happened in this process) and return its exit code."""
    if not args.selftest_cpu:
        have = torch.cuda.device_count()      # does not initialise the GPU on this image
        if have < args.gpus:
            log(f"[bench] --gpus {args.gpus} but only {have} GPU(s) visible")
            print(json.dumps({"error": f"--gpus {args.gpus} needs {args.gpus} GPUs, {have} visible",
                              "n_gpus": args.gpus}), flush=True)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def simulate_world(args):
    """Per-rank compute of the P-rank sharded step on ONE GPU: each rank's share (its rows, edges,
    slab, tiles and support rows) with the collectives left out, graph-captured, timed like the
    real step; then the model: max over ranks + the collectives on the critical path."""
    import hicgat
    from hicgat import dist as hdist
    P = args.simulate_world
    mode = hdist.resolve_mode(args.dist_mode, P)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl = build_workload(args.workload, args.seed, dev)
    rank_ms, rank_med, rank_ms_bare, shards = [], [], [], []
    truth = wl["truth"]
    emulate = args.sim_comm == "emulate"
    sim_coll = {}

    def timed_rank(r, emu):
        torch.manual_seed(0)
        model = hicgat.MODELS[args.model]().to(dev)
        tr = hdist.ShardedTrainer(model, wl["x"], wl["adj"], truth, lr=1e-3, kind=args.loss,
                                  mode=mode, comm=hdist.SimComm(P, r, emulate=emu))
        step = tr.captured(warmup=max(1, args.warmup - 1) if args.warmup >= 2 else max(1, args.warmup))
        if args.warmup >= 2:
            step()       # the last warm-up step: the graph's first replay
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        evs[0].record()
        for k in range(args.steps):
            step()
            evs[k + 1].record()
        torch.cuda.synchronize()
        per = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
        if emu and not sim_coll:
            # the emulated collectives of one eager step, timed on their streams
            hdist.COMM_TIMERS = {}
            tr.step()
            torch.cuda.synchronize()
            sim_coll.update(hdist.comm_report())
            hdist.COMM_TIMERS = None
        return per, tr, step, model

    for r in (range(P) if args.sim_rank is None else [args.sim_rank]):
        per, tr, step, model = timed_rank(r, emulate)
        rank_ms.append(float(np.mean(per)))
        rank_med.append(float(np.median(per)))
        if emulate and not args.no_bare:
            del step, tr, model
            torch.cuda.empty_cache()
            bare, tr, step, model = timed_rank(r, False)
            rank_ms_bare.append(float(np.mean(bare)))
        elif not emulate:
            rank_ms_bare.append(rank_ms[-1])
        shards.append({"rows": tr.local_rows, "nnz": tr.local_nnz, "slab_nnz": getattr(tr, "slab_nnz", None),
                       "tiles": tr.t1 - tr.t0, "support_rows": (tr.s1 - tr.s0) if tr.sf is not None else None})
        log(f"[sim] P={P} rank {r}: {rank_ms[-1]:.4f} ms/step (median {rank_med[-1]:.4f}; without collectives "
            f"{rank_ms_bare[-1] if rank_ms_bare else float('nan'):.4f}) {shards[-1]}")
        del step, tr, model
        torch.cuda.empty_cache()
    n, D = wl["n"], D_FEAT
    coll = {k: hdist.coll_us(kind, nbytes, Pm) for k, (kind, nbytes, Pm) in hdist.MODELED.items()}
    serial_ms = max(rank_ms_bare) + sum(coll.values()) * 1e-3 if rank_ms_bare else None
    # emulated: rank_ms holds the collectives (their time, overlap and CU footprint) -- the model is the
    # slowest rank; left out: the round-4 model, the slowest rank + every collective added serially
    model_ms = max(rank_ms) if emulate else serial_ms
    result = {
        "metric": f"training steps/sec ({args.model}, fwd+loss+bwd+Adam) -- MODELED {P}-GPU step",
        "value": 1e3 / model_ms, "unit": "steps/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": model_ms, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "fp32", "data": "synthetic (power-law Hi-C contacts, 0.1*N(0,1) features, random-init weights seed 0)",
        "config": {"workload": args.workload, "n_nodes": n, "nnz_with_self_loops": wl["adj"].device_nnz,
                   "parallelism": f"dst-row shard x{P} ({mode}), SIMULATED one rank at a time on 1 GPU"},
        "simulated": {"world": P, "mode": mode, "collectives": "emulated" if emulate else "left out",
                      "rank_ms": rank_ms, "rank_median_ms": rank_med,
                      "rank_ms_without_collectives": rank_ms_bare or None,
                      "shards": shards, "collectives_us": coll, "collectives_detail": sim_coll,
                      "serial_model_ms": serial_ms, "model_ms_per_step": model_ms,
                      "assumptions": {"rccl_latency_us": hdist.RCCL_LAT_US, "rccl_bus_GBps": hdist.RCCL_BUS_GBS,
                                      "emulated_collective_workgroups": hdist.SIM_COMM_WGS,
                                      "emulated_collective_threads": hdist.SIM_COMM_THREADS,
                                      "note": "rank_ms measured (graph replay of the rank's share); each collective "
                                              "EMULATED on the stream it is issued on by a kernel holding "
                                              "emulated_collective_workgroups workgroups resident for the modeled "
                                              "time (latency + bytes / bus bandwidth, not measured: 1-GPU box), so "
                                              "overlap with other streams and CU contention are in rank_ms; "
                                              "serial_model_ms = slowest rank without collectives + all modeled "
                                              "collectives added serially (the round-4 model)"}},
    }
    print(json.dumps(result), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="synth-20000", choices=["synth-20000", "synth-2000"])
    ap.add_argument("--loss", default="mse", choices=["mse", "combined", "contrastive"])
    ap.add_argument("--model", default="GATNetSelectiveResidualsUpdated",
                    choices=["GATNetSelectiveResidualsUpdated", "GATNetHeadsChanged3LayersLeakyReLUv2", "Net"],
                    help="the flagship (default), the v2 GAT model or the SAGE baseline Net (SURVEY 8(f) f1); "
                         "N > 1 shards the GAT models only")
    ap.add_argument("--dist-mode", default="auto", choices=["auto", "slab", "xagg", "allgather"],
                    help="N > 1: auto (default: slab at N = 2, xagg from N = 4 -- the faster per world size, "
                         "hicgat.dist.resolve_mode), slab (x replicated, h recomputed per rank, source pass split by "
                         "destination owner -- no h / dout all-gathers), xagg (aggregate-first GATConv: x replicated, "
                         "every GEMM on own rows) or allgather (the RCCL all-gather of h before the layer)")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="one GPU: time each rank's share of a P-rank sharded step, collectives left out")
    ap.add_argument("--sim-rank", type=int, default=None, help="--simulate-world: only this rank (profiling)")
    ap.add_argument("--sim-comm", default="emulate", choices=["emulate", "none"],
                    help="--simulate-world: emulate each collective on its stream (default) or leave them out and "
                         "add them serially (the round-4 model)")
    ap.add_argument("--no-bare", action="store_true",
                    help="--simulate-world: skip the second timing of each rank without the collectives")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5)
    ap.add_argument("--cpu-warmup", type=int, default=2)
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python each step instead of replaying the step as one "
                         "captured hipGraph (the default; at N > 1 the graph holds the RCCL collectives too)")
    ap.add_argument("--graph", action="store_true", help=argparse.SUPPRESS)   # the default; kept for old scripts
    ap.add_argument("--selftest-cpu", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    args.graph = not args.eager and not args.selftest_cpu

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if args.simulate_world:
        return simulate_world(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}")
        sys.exit(2)

    import hicgat
    from hicgat import kernels
    if args.selftest_cpu:
        import torch.distributed as dist
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from cpu_kernels import CpuKernels, torch_tail   # test stand-ins (tests/), never the product
        torch.set_num_threads(1)
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("RANK", "0"), ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("gloo")
        torch_tail(hicgat)
        dev = torch.device("cpu")
        wl = build_selftest_workload(args.seed)
        kern = CpuKernels()
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("nccl", device_id=dev)
        wl = build_workload(args.workload, args.seed, dev)
        kern = None
    torch.manual_seed(0)
    model = hicgat.MODELS[args.model]().to(dev)
    if world > 1 and args.model == "Net":
        raise SystemExit("the sharded step covers the GAT models (Net is the single-GPU f1 baseline)")
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    graph_error = None
    from hicgat import dist as hdist
    if world > 1 or args.selftest_cpu:
        runner = hdist.ShardedTrainer(model, wl["x"], wl["adj"], wl["truth"], lr=1e-3, kind=args.loss, kern=kern,
                                      mode=args.dist_mode)
        wl["truth"] = None                      # each rank keeps only its band (runner.tband)
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        step = runner.step
    else:
        opt = hicgat.FlatAdam(model.flat_parameters(), lr=1e-3)
        stats = torch.empty(12, dtype=torch.float64, device=dev)

        def step():
            return hicgat.train.train_step(model, opt, wl["x"], wl["adj"], wl["truth"], args.loss, stats)

    eager_step = step
    # graph mode: the W untimed warm-up steps are W - 1 eager steps (before the capture) and the graph's
    # first replay (its upload to the device), so the timed region replays a resident graph
    n_eager = max(1, args.warmup - 1) if args.warmup >= 2 else max(1, args.warmup)
    replay_warm = args.warmup >= 2
    # the first eager warm-up step is training step 1 from the seed-0 weights: its loss and forward
    # coordinates are kept for the parity block (the CPU oracle's step 1 on the same workload)
    first = step()
    step1 = {"loss": float(first[0].item()), "coords": first[2].detach().clone()}
    n_eager -= 1
    done_warm = 1
    if args.graph and world > 1:
        try:
            step = runner.captured(warmup=n_eager)   # kernels + RCCL collectives in one graph
        except RuntimeError as exc:   # recorded in the JSON line ("graph": false, "graph_error")
            graph_error = f"{type(exc).__name__}: {exc}"
            log(f"[bench] rank {rank}: GRAPH CAPTURE OF THE SHARDED STEP FAILED ({exc}); timing eager steps")
            sync()
            args.graph = False
            for w in range(done_warm, args.warmup):
                step()
        if args.graph and replay_warm:
            step()
    elif args.graph:
        step = hicgat.graphs.captured_train_step(model, opt, wl["x"], wl["adj"], wl["truth"], args.loss,
                                                 warmup=n_eager)
        if replay_warm:
            step()
    else:
        for w in range(done_warm, args.warmup):
            step()
    sync()
    if world > 1 or args.selftest_cpu:
        torch.distributed.barrier()
    log(f"[bench] warmup done ({args.warmup} steps)")

    kernels.TIMERS = None
    timed_events = dev.type == "cuda"
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if timed_events else []
    sync()
    if world > 1 or args.selftest_cpu:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    if timed_events:
        evs[0].record()
    for k in range(args.steps):
        loss = step()[0]
        if timed_events:
            evs[k + 1].record()
    sync()
    t1 = time.perf_counter()
    if world > 1 or args.selftest_cpu:
        torch.distributed.barrier()
    step_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)] if timed_events else []
    # the reference's loop control (HiC-GNN_main.py:123-132, hicgat.train.train): the same steps, each
    # followed by the host read of the loss and the lossdiff test -- one device -> host sync per step,
    # so the next step's launch waits for it (timed like the headline, reported beside it)
    sync()
    if world > 1 or args.selftest_cpu:
        torch.distributed.barrier()
    old, diffs = 1.0, []
    r0 = time.perf_counter()
    for k in range(args.steps):
        lv = float(step()[0].item())
        diffs.append(abs(old - lv))
        old = lv
    sync()
    loop_s = time.perf_counter() - r0
    if world > 1 or args.selftest_cpu:
        torch.distributed.barrier()
        t = torch.tensor([loop_s], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        loop_s = float(t.item())
    ref_loop = {"value": args.steps / loop_s, "unit": "steps/s", "ms_per_step": 1e3 * loop_s / args.steps,
                "steps": args.steps, "last_lossdiff": diffs[-1],
                "note": "the HiC-GNN_main.py:128 loop: each step's loss read on the host and |old - loss| > thresh "
                        "tested before the next step is launched (graph replay + one D2H sync per step); the "
                        "headline value replays the steps back to back"}
    # per-kernel HIP events: an eager pass of the same length right after the timed region
    kernels.TIMERS = {} if timed_events else None
    sharded = world > 1 or args.selftest_cpu
    if sharded:
        hdist.COMM_TIMERS = {}      # and every collective of the same eager pass, on its stream
    if timed_events or sharded:
        for k in range(args.steps):
            eager_step()
        sync()
    timers, kernels.TIMERS = kernels.TIMERS or {}, None
    comm = None
    if sharded:
        meas = hdist.comm_report()
        hdist.COMM_TIMERS = None
        # the communicator's own rank count: an all-reduce of a one per rank
        one = torch.ones(1, dtype=torch.float32, device=dev if dev.type == "cuda" else "cpu")
        torch.distributed.all_reduce(one)
        pg = torch.distributed.distributed_c10d._get_default_group()
        comm = {"backend": torch.distributed.get_backend(), "world_size": torch.distributed.get_world_size(),
                "process_group_size": pg.size(), "ranks_counted_by_all_reduce": int(round(float(one.item()))),
                "measured_us": {k: {"calls": v["calls"], "avg_us": v["avg_us"], "min_us": v["min_us"],
                                    "bytes": v["bytes"], "kind": v["kind"]} for k, v in meas.items()},
                "modeled_us": {k: v["modeled_us"] for k, v in meas.items()},
                "model_assumptions": {"rccl_latency_us": hdist.RCCL_LAT_US, "rccl_bus_GBps": hdist.RCCL_BUS_GBS},
                "note": "eager pass of the same steps after the timed region: events around each collective on the "
                        "stream it is issued on (gloo: host wall time); a collective's time includes waiting for the "
                        "slowest rank to arrive"}
    elapsed = t1 - t0
    if world > 1 or args.selftest_cpu:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    loss_v = float(loss.item())

    kern_t = {}
    for name, ev in timers.items():
        ms = [a.elapsed_time(b) for a, b in ev]
        kern_t[name] = dict(launches=len(ms), avg_ms=float(np.mean(ms)), total_ms=float(np.sum(ms)))
    n, nnz = wl["n"], wl["adj"].device_nnz
    n_loc = runner.local_rows if sharded else n
    nnz_loc = runner.local_nnz if sharded else nnz
    cands = [k for k in ("gat_agg_fwd", "gat_agg_bwd_dst", "gat_agg_bwd_rows", "gat_agg_bwd_src", "sage_agg",
                         "pairdist_mse_fused") if k in kern_t]
    roof = None
    if cands:
        dom = max(cands, key=lambda k: kern_t[k]["total_ms"])

        def per_launch(k, b):
            """A pass issued as several launches per step: each launch's algorithmic bytes are its share."""
            return b / max(1.0, kern_t[k]["launches"] / args.steps)

        for k in cands:
            b = agg_bytes(k, n, nnz) / world if k == "pairdist_mse_fused" else per_launch(k, agg_bytes(k, n_loc, nnz_loc))
            kern_t[k]["alg_bytes"] = b
            kern_t[k]["alg_GBps"] = b / (kern_t[k]["avg_ms"] * 1e-3) / 1e9
        avg = kern_t[dom]["avg_ms"]
        traffic, src = pmc_traffic(dom, args.workload) if world == 1 else (None, None)
        achieved = traffic / (avg * 1e-3) / 1e9 if traffic else None
        # the gathers' limiter is the Infinity-Cache (MALL) random-row rate of their far edges (the
        # counter bytes are L2 misses, mostly MALL hits): bound "mall", frac vs
        # its 8.6 TB/s; the same bytes against the 8 TB/s HBM peak are kept as hbm_frac
        roof = {"bound": "mall", "kernel": dom,
                "limiter": "L2->CU row-gather rate (near edges) and the Infinity-Cache (MALL) random-row rate "
                           "(far edges); the counter bytes are mostly MALL hits (DESIGN.md section 3)",
                "achieved": achieved, "peak": MALL_GATHER_GBS, "unit": "GB/s",
                "frac": achieved / MALL_GATHER_GBS if achieved else None,
                "hbm_peak": HBM_PEAK_GBS, "hbm_frac": achieved / HBM_PEAK_GBS if achieved else None,
                "traffic": traffic, "traffic_source": src,
                "avg_launch_ms": avg, "launches_per_step": kern_t[dom]["launches"] / args.steps,
                "alg_bytes_per_launch": kern_t[dom]["alg_bytes"], "alg_GBps": kern_t[dom]["alg_GBps"],
                "l2_peak": L2_PEAK_GBS, "l2_frac": kern_t[dom]["alg_GBps"] / L2_PEAK_GBS,
                "note": "achieved: PMC fabric bytes (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) per launch "
                        "/ avg launch time; frac vs the 8.6 TB/s MALL random-row rate, hbm_frac vs 8 TB/s; "
                        "alg_GBps: SURVEY 8(d) no-reuse bytes (every edge reads a whole neighbour row) / time, "
                        "bounded by the L2 (l2_frac), not HBM"}
        tiles = wl["adj"].tiles() if not sharded and dom == "gat_agg_fwd" else None
        if tiles is not None:
            # dense-tile form (a dense contact map): the tile edges are 32x32 . 32x512 products on the
            # fp32 matrix cores, every neighbour row read once per 32 destination rows -- the no-reuse
            # byte model does not apply; the bound is the MFMA rate.  FLOP per launch: two products
            # (out and out2) per tile; the time is the whole call (remainder gather and epilogue too)
            flop = tiles.ntiles * 2 * (2.0 * 32 * 32 * D_FEAT)
            tfs = flop / (avg * 1e-3) / 1e12
            roof.update({"bound": "mfma", "kernel": "gat_agg_fwd (dense-tile form, hicgat_gat_agg_fwd_tiled)",
                         "achieved": tfs, "peak": MFMA_F32_TFS, "unit": "TFLOP/s", "frac": tfs / MFMA_F32_TFS,
                         "traffic": None, "traffic_source": None, "flop_per_launch": flop,
                         "dense_tiles": tiles.ntiles, "edges_in_tiles": tiles.n_dense, "l2_frac": None,
                         "note": "dense-tile aggregation: achieved = tile MFMA FLOP (2 products x 2*32*32*512 per "
                                 "tile) / avg time of the whole call (incl. the remainder gather and epilogue); "
                                 "alg_GBps is the no-reuse byte model, which tiles (32-row reuse) do not follow"})

    result = {
        "metric": f"training steps/sec ({args.model}, fwd+loss+bwd+Adam)",
        "value": args.steps / elapsed,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "median_ms_per_step": float(np.median(step_ms)) if step_ms else None,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (power-law Hi-C contacts, 0.1*N(0,1) features, random-init weights seed 0)"
                if not args.selftest_cpu else "SELFTEST: CPU gloo ranks + torch stand-in kernels, 400 nodes -- not a measurement",
        "graph": bool(args.graph),
        "model": args.model,
        "config": {"workload": args.workload if not args.selftest_cpu else "selftest-400",
                   "n_nodes": n, "nnz_with_self_loops": nnz, "d": D_FEAT, "heads": HEADS,
                   "loss": args.loss,
                   "parallelism": (f"dst-row shard x{world} (nnz-balanced, {runner.mode})" if sharded else "single"),
                   "gemm": "fp32 MFMA" if not args.selftest_cpu else "cpu stand-in"},
        "final_loss": loss_v,
        "reference_loop": ref_loop,
        "roofline": roof,
        "gemm": gemm_block(args.workload, kern_t) if not args.selftest_cpu else None,
        "kernels": kern_t,
    }
    if comm is not None:
        result["collectives"] = comm
    if sharded:
        result["shard"] = {"mode": runner.mode, "rows_per_rank": [int(v) for v in runner.plan.counts],
                           "nnz_per_rank": [int(v) for v in runner.plan.nnz]}
    if graph_error is not None:
        result["graph_error"] = graph_error
    if rank == 0 and world == 1 and not args.selftest_cpu and not args.no_cpu_baseline \
            and args.model == "GATNetSelectiveResidualsUpdated":
        log("[bench] cpu baseline (oracle) ...")
        cb = cpu_baseline(wl, args.seed, steps=args.cpu_steps, warmup=args.cpu_warmup)
        result["parity"] = parity_block(step1, cb.pop("step1"))
        result["cpu_baseline"] = cb
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1 or args.selftest_cpu:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
