"""Per-kernel timing on the synth-20000 workload (HIP events, interleaved rounds).

  python tools/kbench.py [--libs a.so,b.so] [--reps 20] [--workload synth-20000]

Loads each library build (same C ABI) in turn via ctypes, runs every kernel of the training step
on identical inputs and prints avg/min ms and algorithmic GB/s (bench.agg_bytes) per kernel."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--workload", default="synth-20000")
    ap.add_argument("--only", default="", help="comma-separated job-name substrings to run")
    a = ap.parse_args()
    import bench
    import hicgat
    from hicgat import _lib, kernels
    dev = torch.device("cuda", 0)
    wl = bench.build_workload(a.workload, 0, dev)
    n, adj, truth, x = wl["n"], wl["adj"], wl["truth"], wl["x"]
    nnz = adj.device_nnz
    torch.manual_seed(0)
    model = hicgat.GATNetSelectiveResidualsUpdated().to(dev)
    conv = model.conv
    W, al, ar, b = conv.lin_l.weight.detach(), conv.att_l.detach(), conv.att_r.detach(), conv.bias.detach()
    K0 = kernels.HipKernels()
    h, a_s, a_d = K0.linear_att(x, W, al, ar)
    out = torch.empty_like(h)
    rs = torch.zeros(n, 8, device=dev)
    out2 = torch.empty_like(h)
    K0.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, 1, out, out2, rs)
    dout = torch.randn_like(h) * 1e-3
    dh = torch.empty_like(h)
    da = torch.empty_like(a_s)
    coords = torch.randn(n, 3, device=dev)
    stats = torch.empty(12, dtype=torch.float64, device=dev)
    loss = torch.empty((), device=dev)
    dc = torch.empty_like(coords)
    flat = torch.randn(601600, device=dev)
    g = torch.randn_like(flat)
    m = torch.zeros_like(flat)
    v = torch.zeros_like(flat)
    Wa = model.densea.weight.detach()
    ba = model.densea.bias.detach()
    ya = torch.empty(n, 256, device=dev)
    dxa = torch.empty(n, 512, device=dev)
    cs = torch.empty(512, device=dev)
    lns = torch.rand(n, 2, device=dev)
    g256, g256b, g256c = torch.randn(256, device=dev), torch.empty(256, device=dev), torch.empty(256, device=dev)
    ya2 = torch.empty(n, 256, device=dev)
    libs = [s for s in a.libs.split(",") if s] or [_lib.LIB_PATH]
    _tiles = {}

    def tiles():   # the dense-tile split at HICGAT_TILE_MIN (64 when tiling is off by default)
        if not _tiles:
            _tiles["t"] = hicgat.graph.build_tiles(adj.rowptr32, adj.col32, 0, n, n, hicgat.graph.TILE_MIN or 64)
        return _tiles["t"]
    kset = []
    for path in libs:
        lib = ctypes.CDLL(path)
        for name, (res, args) in _lib.SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        K = kernels.HipKernels.__new__(kernels.HipKernels)
        K.lib = lib
        K.gemm_impl = 1              # fp32 MFMA
        kset.append((os.path.basename(path), K))
    jobs = {
        "gat_linear_att": lambda K: K.linear_att(x, W, al, ar),
        "gat_agg_fwd": lambda K: K.agg_fwd(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, out, rs),
        "gat_agg_fwd_train": lambda K: K.agg_fwd_act(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, b, 0.2, 1, out,
                                                     out2, rs),
        "gat_agg_bwd_dst": lambda K: K.agg_bwd_dst(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, dout, 0.2, rs),
        "gat_agg_bwd_rows": lambda K: K.agg_bwd_rows(0, n, 1, dout, out, b, out2, dh, rs),
        "gat_agg_bwd_src": lambda K: K.agg_bwd_src(adj.rowptr32, adj.col32, 0, n, h, a_s, a_d, rs, dout, al, ar,
                                                   0.2, dh, da),
        "param_grad": lambda K: K.param_grad(h, dout, da, rs, 2),
        "pairdist_mse_fused": lambda K: K.fused_loss(coords, truth.buf, n, 0, 0, -1, stats, loss, dc),
        "pairdist_combined": lambda K: K.fused_loss(coords, truth.buf, n, 1, 0, -1, stats, loss, dc),
        "pairdist_support": lambda K: K.fused_loss_support(coords, truth.support, n, 0, stats, loss, dc),
        "pairdist_support_combined": lambda K: K.fused_loss_support(coords, truth.support, n, 1, stats, loss, dc),
        "gat_agg_fwd_tiled": lambda K: K.agg_fwd_tiled(adj.rowptr32, adj.col32, tiles(), h, a_s, a_d, b, 0.2, 1, out,
                                                       out2, rs),
        "gat_agg_bwd_src_tiled": lambda K: K.agg_bwd_src_tiled(tiles(), h, a_s, a_d, rs, dout, al, ar, 0.2, dh, da),
        "colsum_20000x512": lambda K: K.colsum(out, cs),
        "ln_bwd_256": lambda K: K.ln_relu_res_bwd(ya, ya, lns, g256, g256, ya2, g256b, g256c),
        "adam": lambda K: K.adam(flat, g, m, v, flat.numel(), 1e-3, 0.9, 0.999, 1e-8, 1),
        "gemm_dw_512x512": lambda K: hicgat.ops.weight_grad(K, dh, x),
        "gemm_fwd_densea": lambda K: K.gemm(0, 0, n, 256, 512, out, Wa, ya, bias=ba),
        "gemm_dx_densea": lambda K: K.gemm(0, 1, n, 512, 256, ya, Wa, dxa),
        "gemm_dw_densea": lambda K: hicgat.ops.weight_grad(K, ya, out),
        "torch_dw_densea": lambda K: ya.t().mm(out),
        "torch_dw_512x512": lambda K: dh.t().mm(x),   # the library GEMM (hipBLASLt) on the same shape
        "torch_fwd_densea": lambda K: torch.nn.functional.linear(out, Wa, ba),
    }
    if a.only:
        keys = [k.strip() for k in a.only.split(",") if k.strip()]
        jobs = {k: v for k, v in jobs.items() if any(x in k for x in keys)}
    res = {}
    for r in range(a.rounds):
        for lname, K in kset:
            for jname, fn in jobs.items():
                fn(K)
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn(K)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((lname, jname), []).append(e0.elapsed_time(e1) / a.reps)
    for (lname, jname), ts in res.items():
        alg = ""
        base = jname.split("@")[0]
        if base in ("gat_agg_fwd", "gat_agg_fwd_train", "gat_agg_bwd_dst", "gat_agg_bwd_rows", "gat_agg_bwd_src",
                    "pairdist_mse_fused", "pairdist_combined"):
            kb = {"pairdist_combined": "pairdist_mse_fused", "gat_agg_fwd_train": "gat_agg_fwd"}.get(base, base)
            alg = f"{bench.agg_bytes(kb, n, nnz) / (min(ts) * 1e-3) / 1e9:9.0f} GB/s alg"
        print(f"{lname:28s} {jname:22s} med {np.median(ts):8.4f} ms  min {min(ts):8.4f} ms  {alg}", flush=True)


if __name__ == "__main__":
    main()
