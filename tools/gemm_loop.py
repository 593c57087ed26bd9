"""Run one GEMM shape repeatedly (for rocprofv3 PMC passes): python tools/gemm_loop.py [fwd|dx] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd")]
import torch  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    import hicgat
    K = hicgat.kernels.default()
    dev = "cuda"
    m, n, k = 20000, 512, 512
    x = torch.randn(m, k, device=dev)
    w = torch.randn(n, k, device=dev)
    y = torch.empty(m, n, device=dev)
    for _ in range(reps):
        if kind == "fwd":
            K.gemm(0, 0, m, n, k, x, w, y)
        else:
            K.gemm(0, 1, m, n, k, x, w, y)
    torch.cuda.synchronize()
    print("ok", float(y[0, 0]))


if __name__ == "__main__":
    main()
