"""fp32 GEMM rates of the step's big node-row GEMMs: this library's kernels against torch.mm
(hipBLASLt / rocBLAS) on the same shapes -- a diagnostic for whether a library GEMM would serve
better (GPU box: python tools/gemm_lib_bench.py)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd")]


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from hicgat import kernels, ops
    torch.backends.cuda.matmul.allow_tf32 = False
    K = kernels.default()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M, F = 20000, 512
    x = torch.randn(M, F, device=dev)
    W = torch.randn(F, F, device=dev) * 0.05
    dy = torch.randn(M, F, device=dev)
    out = torch.empty(M, F, device=dev)
    dW = torch.empty(F, F, device=dev)
    fl = 2.0 * M * F * F
    rows = []
    t = timeit(lambda: K.gemm(0, 0, M, F, F, x, W, out))
    rows.append(("fwd  x W^T  [20000x512]x[512x512]  hicgat", t))
    t = timeit(lambda: torch.mm(x, W.t(), out=out))
    rows.append(("fwd  x W^T                         torch.mm", t))
    t = timeit(lambda: ops.weight_grad(K, dy, x, out=dW))
    rows.append(("dW   dy^T x [512x20000]x[20000x512] hicgat", t))
    t = timeit(lambda: torch.mm(dy.t(), x, out=dW))
    rows.append(("dW   dy^T x                        torch.mm", t))
    for name, us in rows:
        print(f"{name:48s} {us:8.1f} us  {fl / us * 1e-6:6.1f} TF")


if __name__ == "__main__":
    main()
