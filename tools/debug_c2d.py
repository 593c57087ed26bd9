"""Diagnose hicgat_cont2dist vs torch CPU: count and show the first differing elements."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "hic-gnn_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import hicgat  # noqa: E402
from conftest import load_golden  # noqa: E402
from oracle import graph as og  # noqa: E402

g = load_golden("graph_chr19_1mb.npz")
y = torch.tensor(g["matrix"], dtype=torch.float64)
y.fill_diagonal_(0)
for f in (0.5, 1.0):
    ref = og.cont2dist(y.clone(), f)
    got = hicgat.cont2dist(y.cuda(), f).cpu()
    diff = (ref != got)
    print(f"factor {f}: {int(diff.sum())} / {diff.numel()} differ")
    idx = diff.nonzero()[:5]
    for i, j in idx.tolist():
        a, b = ref[i, j].item(), got[i, j].item()
        ua = np.float64(a).view(np.int64)
        ub = np.float64(b).view(np.int64)
        r = (1 / y[i, j]).item()
        print(f"  ({i},{j}) y={y[i,j].item()!r} ref={a!r} got={b!r} ulps={ub - ua} sqrt(1/y)={np.sqrt(r)!r}")
    mx_ref = torch.max(torch.nan_to_num((1 / y) ** f, posinf=0)).item()
    print("  max ref", mx_ref)
# raw sqrt check through factor 0.5 on a 1 x n "matrix" is not possible (N x N); use n = 2000 randoms
n = 1500
yy = torch.rand(n, n, dtype=torch.float64) * 100 + 0.01
ref = og.cont2dist(yy.clone(), 0.5)
got = hicgat.cont2dist(yy.cuda(), 0.5).cpu()
print("random 0.5:", int((ref != got).sum()), "differ of", n * n)
raw_ref = torch.sqrt(1 / yy)
print("  max |got*max - sqrt(1/y)| ulp-ish:", float(((got - ref).abs() / ref.abs().clamp_min(1e-300)).max()))
