"""CPU restatement of the reference's Knight-Ruiz normalisation (TEST INFRASTRUCTURE ONLY).

Reference: ``r_utils.R:1-93`` ``KRnorm``, run by ``normalize.R:1-11`` as an ``Rscript``
subprocess from ``HiC-GNN_main.py:85`` (R is not installed in this image, so the R code cannot be
run here).  Restated in numpy float64, statement by statement,
keeping the reference's behaviour where it differs from textbook KR:

* ``zeros = unique(which(colSums(A) == 0), which(rowSums(A) == 0))`` (:3): the second argument of
  R's ``unique`` is ``incomparables``, so only the zero COLUMNS are collected (the matrices are
  symmetric, so rows and columns agree anyway); those rows and columns are dropped (:6-7);
* NAs are set to 0 for the iteration and put back at the end (:13-15, :76-80);
* the inner CG loop assigns ``Z = rk/v`` (:60) where ``z`` was meant, so ``z`` keeps its k == 1
  value ``rk/v`` for the whole inner loop (used by ``rho_km1 = t(rk) %*% z`` and ``p = z + beta p``);
* the boundary tests (:46-57) and the eta update (:65-71) as written;
* ``round(result, digits = 6)`` (:89), the value ``write.table`` saves and ``np.loadtxt`` reads
  back (HiC-GNN_main.py:89): the nearest double to the 6-decimal number, i.e. rint(x*1e6)/1e6.

Pinned by the reference's ``Outputs/`` files: this restatement + the reference ``convert_to_matrix``
/ ``cont2dist`` + Spearman on the coordinates of ``Outputs/*_structure.pdb`` reproduces the logged
dSCC (tests/test_oracle_golden.py::test_kr_reproduces_logged_dscc).
"""
import numpy as np

TOL, DELTA, DELTA_UP, G, ETAMAX = 1e-6, 0.1, 3.0, 0.9, 0.1


def krnorm(A, return_info=False):
    """``KRnorm(A)`` (r_utils.R:1-93) -> (normed matrix without the zero rows/cols, kept index).

    ``A`` is a square float64 array (NaN allowed).  The kept index lists the rows/columns of A
    that survive the zero-column removal (R keeps them as dimnames)."""
    A = np.array(A, dtype=np.float64)
    with np.errstate(invalid="ignore"):
        cs = A.sum(axis=0)
    zeros = np.unique(np.nonzero(cs == 0)[0])                      # :3 (rowSums are `incomparables`)
    keep = np.setdiff1d(np.arange(A.shape[0]), zeros)
    A = A[np.ix_(keep, keep)]                                      # :6-7
    na = np.isnan(A)                                               # :13-15
    A[na] = 0.0
    n = A.shape[0]
    e = np.ones(n)
    stop_tol = TOL * 0.5
    eta = ETAMAX
    x = e.copy()
    rt = TOL ** 2
    v = x * (A @ x)
    rk = 1.0 - v
    rho_km1 = float(rk @ rk)
    rout = rho_km1
    rold = rout
    outer, mvp = 0, 0
    z = p = None
    while rout > rt:                                               # :27 outer iteration
        outer += 1
        k = 0
        y = e.copy()
        innertol = max(eta ** 2 * rout, rt)
        while rho_km1 > innertol:                                  # :30 inner CG
            k += 1
            if k == 1:
                z = rk / v
                p = z
                rho_km1 = float(rk @ z)
            else:
                beta = rho_km1 / rho_km2
                p = z + beta * p
            w = x * (A @ (x * p)) + v * p                          # :42
            alpha = rho_km1 / float(p @ w)
            ap = alpha * p
            ynew = y + ap
            if ynew.min() <= DELTA:                                # :47
                ind = ap < 0
                gamma = np.min((DELTA - y[ind]) / ap[ind])
                y = y + gamma * ap
                break
            if ynew.max() >= DELTA_UP:                             # :53
                ind = ynew > DELTA_UP
                gamma = np.min((DELTA_UP - y[ind]) / ap[ind]) if ind.any() else np.inf
                y = y + gamma * ap
                break
            y = ynew
            rk = rk - alpha * w
            rho_km2 = rho_km1
            # :60 `Z = rk/v` -- assigns a new variable; z keeps its k == 1 value
            rho_km1 = float(rk @ z)
        x = x * y                                                  # :63
        v = x * (A @ x)
        rk = 1.0 - v
        rho_km1 = float(rk @ rk)
        rout = rho_km1
        mvp += k + 1
        rat = rout / rold                                          # :68
        rold = rout
        res_norm = np.sqrt(rout)
        eta_o = eta
        eta = G * rat
        if G * eta_o ** 2 > 0.1:
            eta = max(eta, G * eta_o ** 2)
        eta = max(min(eta, ETAMAX), stop_tol / res_norm)
    result = x[:, None] * A * x[None, :]                           # :74 t(t(x*A)*x)
    result[na] = np.nan
    result = round6(result)                                        # :89
    if return_info:
        return result, keep, dict(outer=outer, mvp=mvp, x=x)
    return result, keep


def round6(a):
    """R's round(x, 6) as saved by write.table and parsed by np.loadtxt: the double nearest to the
    6-decimal value (rint(x * 1e6) / 1e6; q / 1e6 is a correctly rounded division)."""
    return np.rint(a * 1e6) / 1e6
