"""Knight-Ruiz normalisation on the GPU.

``KRnorm(A)`` mirrors ``r_utils.R:1-93`` (run by ``normalize.R`` as an ``Rscript`` subprocess at
``HiC-GNN_main.py:85``; the reference hands the result over through ``Data/*_KR_normed.txt``).
The O(N^2) work -- every matrix-vector product and the final scaling + 6-digit rounding -- runs in
``libhicgat.so`` (``hicgat_kr_matvec`` / ``hicgat_kr_scale``, csrc/kr.hip); the O(N) CG bookkeeping
of the R code runs here on device vectors, statement by statement, including its quirks:

* only zero COLUMNS are removed (``unique(a, b)`` treats ``b`` as ``incomparables``, :3);
* NA -> 0 for the iteration, NA restored in the result (:13-15, :76-80);
* ``Z = rk/v`` at :60 never updates ``z`` (the k == 1 value is used for the whole inner loop);
* ``round(result, 6)`` (:89), the value ``write.table`` writes and ``np.loadtxt`` reads back.

The loop conditions are host decisions exactly as in R (one device->host read per test).
"""
import torch

from . import _lib

TOL, DELTA, DELTA_UP, G, ETAMAX = 1e-6, 0.1, 3.0, 0.9, 0.1
P = _lib.ptr


def _matvec(A, x, p, v=None):
    out = torch.empty_like(x)
    _lib.check(_lib.lib().hicgat_kr_matvec(P(A), A.stride(0), A.shape[0], P(x), P(p), P(v), P(out),
                                           _lib.stream(A.device)), "hicgat_kr_matvec")
    return out


def KRnorm(A, device="cuda", return_info=False):
    """r_utils.R KRnorm on the GPU.  ``A``: square float64 matrix (numpy or tensor, NaN allowed).
    Returns ``(normed, keep)``: the balanced, 6-digit-rounded float64 matrix on ``device`` without
    the zero columns/rows, and the kept row indices (R's dimnames)."""
    A = torch.as_tensor(A, dtype=torch.float64).to(device)
    if A.dim() != 2 or A.shape[0] != A.shape[1]:
        raise ValueError("KRnorm needs a square matrix")
    cs = A.sum(0)
    keep = torch.nonzero(cs != 0).flatten()          # :3 zero columns (NaN sums are kept, as in R)
    if keep.numel() != A.shape[0]:
        A = A.index_select(0, keep).index_select(1, keep).contiguous()   # :6-7
    A = A.contiguous()
    n = A.shape[0]
    e = torch.ones(n, dtype=torch.float64, device=A.device)
    stop_tol = TOL * 0.5
    eta = ETAMAX
    x = e.clone()
    rt = TOL ** 2
    v = _matvec(A, x, e)                              # v = x * (A %*% x)
    rk = 1.0 - v
    rho_km1 = float(rk @ rk)
    rout, rold = rho_km1, rho_km1
    outer = mvp = 0
    z = p = None
    rho_km2 = None
    while rout > rt:
        outer += 1
        k = 0
        y = e.clone()
        innertol = max(eta ** 2 * rout, rt)
        while rho_km1 > innertol:
            k += 1
            if k == 1:
                z = rk / v
                p = z
                rho_km1 = float(rk @ z)
            else:
                beta = rho_km1 / rho_km2
                p = z + beta * p
            w = _matvec(A, x, p, v)                   # x * (A %*% (x*p)) + v*p
            alpha = rho_km1 / float(p @ w)
            ap = alpha * p
            ynew = y + ap
            if float(ynew.min()) <= DELTA:
                ind = ap < 0
                gamma = float(((DELTA - y[ind]) / ap[ind]).min())
                y = y + gamma * ap
                break
            if float(ynew.max()) >= DELTA_UP:
                ind = ynew > DELTA_UP
                gamma = float(((DELTA_UP - y[ind]) / ap[ind]).min()) if bool(ind.any()) else float("inf")
                y = y + gamma * ap
                break
            y = ynew
            rk = rk - alpha * w
            rho_km2 = rho_km1
            rho_km1 = float(rk @ z)                   # :60 -- z is never refreshed
        x = x * y
        v = _matvec(A, x, e)
        rk = 1.0 - v
        rho_km1 = float(rk @ rk)
        rout = rho_km1
        mvp += k + 1
        rat = rout / rold
        rold = rout
        res_norm = rout ** 0.5
        eta_o = eta
        eta = G * rat
        if G * eta_o ** 2 > 0.1:
            eta = max(eta, G * eta_o ** 2)
        eta = max(min(eta, ETAMAX), stop_tol / res_norm)
    out = torch.empty_like(A)
    _lib.check(_lib.lib().hicgat_kr_scale(P(A), A.stride(0), n, P(x), P(out), out.stride(0),
                                          _lib.stream(A.device)), "hicgat_kr_scale")
    if return_info:
        return out, keep, dict(outer=outer, mvp=mvp, x=x)
    return out, keep

