"""Debug the 160x128 tall GEMM: error pattern vs torch on small shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd")]
import torch  # noqa: E402


def main():
    import hicgat
    K = hicgat.kernels.default()
    dev = "cuda"
    for (m, n, k, bk) in [(1024, 128, 16, 0), (1024, 128, 32, 0), (1024, 128, 64, 0), (1024, 256, 512, 0),
                          (1024, 128, 16, 1), (1024, 128, 64, 1), (20000, 256, 512, 0)]:
        torch.manual_seed(0)
        x = torch.randn(m, k, device=dev)
        if bk == 0:
            w = torch.randn(n, k, device=dev)
            y = K.gemm(0, 0, m, n, k, x, w, torch.zeros(m, n, device=dev))
            ref = x.double() @ w.double().t()
        else:
            w = torch.randn(k, n, device=dev)
            y = K.gemm(0, 1, m, n, k, x, w, torch.zeros(m, n, device=dev))
            ref = x.double() @ w.double()
        err = (y.double() - ref).abs()
        rel = float(err.max() / ref.abs().max())
        bad = (err > 1e-4 * ref.abs().max())
        print(f"m={m} n={n} k={k} bkm={bk}: rel {rel:.3e}, bad {int(bad.sum())}/{bad.numel()}")
        if bad.any():
            r, c = torch.nonzero(bad, as_tuple=True)
            print("  rows%160 hist:", torch.bincount(r % 160, minlength=160)[:40].tolist())
            print("  cols%128 hist:", torch.bincount(c % 128, minlength=128)[:40].tolist())
            print("  first bad:", [(int(a), int(b)) for a, b in zip(r[:8], c[:8])])
            # is the bad value equal to some other reference entry (permutation)?
            i, j = int(r[0]), int(c[0])
            v = float(y[i, j])
            hits = torch.nonzero((ref[i] - v).abs() < 1e-3 * ref.abs().max())
            print("  y[i,j]", v, "ref[i,j]", float(ref[i, j]), "matches ref[i, cols]", hits.flatten()[:5].tolist())


if __name__ == "__main__":
    main()
