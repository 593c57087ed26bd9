"""Measurement of the once-per-run rows of SURVEY.md section 8(f) (f2 KR normalisation, f3
Procrustes alignment) on MI355X, with the CPU oracle timed on the same input.

  python tools/bench_aux.py [--n 20000] [--cpu-n 4000]

Prints one JSON line: for KR the GPU time of the whole KRnorm (HIP matvec / scale kernels + the
device CG bookkeeping, host loop tests included) on a dense synthetic Hi-C matrix, the number of
matrix-vector products, the matvec kernel's achieved HBM GB/s (8 N^2 bytes per product) and the
oracle's time on a smaller matrix (numpy float64, all host threads); for Procrustes the device time
of domain_alignment at F = 512.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def dense_contacts(n, seed, device="cuda"):
    """The synth-20000 contact matrix (1 % power-law density, float64) as KRnorm's input."""
    from hicgat import synth
    i, j, c = synth.contact_pairs(n, density=0.01, seed=seed)
    return synth.dense_contacts(n, i, j, c, device=device)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--cpu-n", type=int, default=3000)
    a = ap.parse_args()
    import hicgat
    from oracle import kr as okr
    res = {"metric": "aux once-per-run rows (f2 KR, f3 Procrustes)"}
    A = dense_contacts(a.n, 0)
    torch.cuda.synchronize()
    hicgat.kr.KRnorm(A[:256, :256].clone())            # warm up (library load, kernels)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, keep, info = hicgat.kr.KRnorm(A, return_info=True)
    torch.cuda.synchronize()
    t_gpu = time.perf_counter() - t0
    x = torch.ones(a.n, dtype=torch.float64, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        hicgat.kr._matvec(A, x, x, x)
    e1.record()
    torch.cuda.synchronize()
    mv_ms = e0.elapsed_time(e1) / 10
    del out
    Ac = dense_contacts(a.cpu_n, 0, device="cpu").numpy()
    t0 = time.perf_counter()
    _, _, cinfo = okr.krnorm(Ac, return_info=True)
    t_cpu = time.perf_counter() - t0
    res["kr"] = {"n": a.n, "gpu_s": t_gpu, "matvecs": info["mvp"] + 1, "outer": info["outer"],
                 "matvec_ms": mv_ms, "matvec_GBps": 8.0 * a.n * a.n / (mv_ms * 1e-3) / 1e9,
                 "cpu_baseline": {"n": a.cpu_n, "s": t_cpu, "matvecs": cinfo["mvp"] + 1, "kind": "port",
                                  "cores": os.cpu_count(), "note": "oracle/kr.py numpy float64 (BLAS threads)"}}
    rng = np.random.default_rng(0)
    l1 = np.stack([np.arange(0, 2000) * 1000000, np.arange(0, 2000) * 1000000, np.ones(2000)], 1)
    l2 = np.stack([np.arange(0, 4000) * 500000, np.arange(0, 4000) * 500000, np.ones(4000)], 1)
    e1 = rng.standard_normal((2000, 512)).astype(np.float32)
    e2 = rng.standard_normal((4000, 512)).astype(np.float32)
    hicgat.align.domain_alignment(l1, l2, e1, e2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hicgat.align.domain_alignment(l1, l2, e1, e2)
    torch.cuda.synchronize()
    res["procrustes"] = {"bins_1mb": 2000, "bins_500kb": 4000, "F": 512, "gpu_s": time.perf_counter() - t0}
    # f4: node2vec with the reference's call (HiC_GAT_generalize_directly.py:153-154) on chr19 1 mb
    # (the config-1 graph) and on a synthetic 2000-locus Hi-C matrix
    from conftest import load_golden
    from hicgat import embed, synth
    n2v = {}
    for name, mat in (("chr19_1mb", load_golden("graph_chr19_1mb.npz")["matrix"].copy()),
                      ("synth2000_1pct", dense_contacts(2000, 0, device="cpu").numpy())):
        embed.node2vec(mat[:32, :32], dimensions=64, walk_length=10, num_walks=2, epochs=1)   # warm up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        walks = embed.random_walks(mat)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        embed.skipgram(walks, mat.shape[0])
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        steps = int((walks >= 0).sum().item())
        n2v[name] = {"n": int(mat.shape[0]), "walks": int(walks.shape[0]), "walk_steps": steps,
                     "walks_s": t1 - t0, "skipgram_5_epochs_s": t2 - t1,
                     "note": "dimensions 512, walk_length 150, num_walks 50, p 1.75, q 0.4, window 25, 5 epochs"}
    res["node2vec"] = n2v
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
