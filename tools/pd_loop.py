"""Run only the fused distance/MSE loss on the synth-20000 truth (for rocprofv3 PMC passes):
python tools/pd_loop.py [reps] [--lib path]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd")]

import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    import bench
    from hicgat import kernels
    dev = torch.device("cuda", 0)
    wl = bench.build_workload("synth-20000", 0, dev)
    n, truth = wl["n"], wl["truth"]
    coords = torch.randn(n, 3, device=dev)
    stats = torch.empty(12, dtype=torch.float64, device=dev)
    loss = torch.empty((), device=dev)
    dc = torch.empty_like(coords)
    K = kernels.default()
    for _ in range(reps):
        K.fused_loss(coords, truth.buf, n, 0, 0, -1, stats, loss, dc)
    torch.cuda.synchronize()
    print("loss", float(loss))


if __name__ == "__main__":
    main()
