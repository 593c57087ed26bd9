"""Generate ``dscc_band_chr19_1mb.npz``: the oracle's dSCC on GM12878 chr19 1 mb after a fixed
K = 3000 steps of the HiC-GNN_main.py loop (HiC-GNN_main.py:92-139: KR normalise, load_input,
cont2dist(y, 0.5), Adam lr 1e-3, get_model, Spearman of the upper-triangle distances), run at 1, 2,
4 and 8 CPU threads.  The thread count changes torch's summation order and the fixed-K training is
chaotic, so the spread of these four runs is the oracle's own noise floor; the GPU
test (tests/test_gpu_parity.py::test_dscc_chr19_1mb_k3000_matches_oracle) compares the device
result with the 1-thread value and prints that floor beside the difference.

Test infrastructure only (it runs the CPU oracle under oracle/).  Inputs: the committed fixtures
graph_chr19_1mb.npz (the reference's contact matrix) and model_GATNetSelectiveResidualsUpdated.npz
(512-d features; node2vec is absent).

    python tests/golden/make_dscc_band.py      # ~5 min on 8 cores

``--seeds`` runs the same pipeline at 1 thread for initial-weight seeds 0..7 (one process per seed)
and writes ``dscc_seeds_chr19_1mb.npz``: the summation-order-robust protocol of the GPU test (the
MEDIAN dSCC over the eight seeds, which both of the device's aggregation forms must reproduce within
+-0.005; a mean over four seeds moved by 1.3e-2 when one device seed fell into another basin).

``--features n2v`` uses the node2vec embedding ``n2v_chr19_1mb.npz`` (tests/golden/make_n2v_chr19.py,
this repo's GPU node2vec with the reference's parameters) instead of the fixture's random features
and writes ``dscc_band_chr19_1mb_n2v.npz`` (BASELINE configs[0]: 512-d node2vec).
"""
import os
import platform
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import gat as og  # noqa: E402
from oracle import graph as ogr  # noqa: E402
from oracle import kr as okr  # noqa: E402
from oracle import loop as ol  # noqa: E402

K = 3000
THREADS = (1, 2, 4, 8)
SEEDS = tuple(range(8))


def _run(th, sd, d, radj, truth):
    og.CDIST_MODE = "donot_use_mm_for_euclid_dist"
    try:
        torch.set_num_threads(th)
        torch.manual_seed(sd)
        ref = og.GATNetSelectiveResidualsUpdated()
        t0 = time.time()
        hist = ol.train(ref, d["x"], radj, truth, steps=K)
        with torch.no_grad():
            rho = ol.dscc(ref.get_model(d["x"], radj), truth)
        print(f"threads {th} seed {sd}: dSCC {rho:.6f}, loss {hist[-1]:.6e} ({time.time() - t0:.0f} s)", flush=True)
        return rho, hist[-1]
    finally:
        og.CDIST_MODE = "use_mm_for_euclid_dist_if_necessary"


def main():
    with np.load(os.path.join(HERE, "graph_chr19_1mb.npz"), allow_pickle=False) as z:
        a = np.array(z["matrix"], dtype=np.float64)
    feat = sys.argv[sys.argv.index("--features") + 1] if "--features" in sys.argv else "fixture"
    n2v = feat.startswith("n2v")
    # n2v: n2v_chr19_1mb.npz (seed 42); n2v43: n2v_chr19_1mb_s43.npz (the second node2vec seed)
    src = {"fixture": "model_GATNetSelectiveResidualsUpdated.npz", "n2v": "n2v_chr19_1mb.npz",
           "n2v43": "n2v_chr19_1mb_s43.npz"}[feat]
    out_name = {"fixture": "dscc_band_chr19_1mb.npz", "n2v": "dscc_band_chr19_1mb_n2v.npz",
                "n2v43": "dscc_band_chr19_1mb_n2v43.npz"}[feat]
    with np.load(os.path.join(HERE, src), allow_pickle=False) as z:
        x = np.asarray(z["x"], dtype=np.float32)
    np.fill_diagonal(a, 0)
    normed, keep = okr.krnorm(a.copy())
    x = x[np.asarray(keep)] if len(keep) != len(x) else x
    d = ogr.load_input(normed.copy(), x)
    truth = ogr.cont2dist(d["y"], 0.5)
    radj = (torch.tensor(d["rowptr"]), torch.tensor(d["col"]))
    seeds_mode = "--seeds" in sys.argv
    runs = [(1, sd) for sd in SEEDS] if seeds_mode else [(th, 0) for th in THREADS]
    if seeds_mode:
        # 1-thread runs: one process per seed (same arithmetic as running them one after another)
        import multiprocessing as mpr
        with mpr.get_context("fork").Pool(min(len(runs), os.cpu_count() or 1)) as pool:
            res = pool.starmap(_run, [(th, sd, d, radj, truth) for th, sd in runs])
    else:
        res = [_run(th, sd, d, radj, truth) for th, sd in runs]
    dscc = [r[0] for r in res]
    loss = [r[1] for r in res]
    if seeds_mode:
        np.savez(os.path.join(HERE, "dscc_seeds_chr19_1mb.npz"), steps=np.int64(K), seeds=np.array(SEEDS),
                 dscc=np.array(dscc), loss=np.array(loss), torch=np.array(torch.__version__),
                 cpu=np.array(platform.processor() or platform.machine()))
        return
    np.savez(os.path.join(HERE, out_name), steps=np.int64(K), threads=np.array(THREADS),
             dscc=np.array(dscc), loss=np.array(loss), torch=np.array(torch.__version__),
             cpu=np.array(platform.processor() or platform.machine()))


if __name__ == "__main__":
    main()
