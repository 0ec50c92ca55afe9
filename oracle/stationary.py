"""CPU ORACLE (test infrastructure only) -- build-defined stationary extensions.

SURVEY.md §2 lists three extensions that ``north_star`` requires but the reference does
not implement (E1 GE bisection on r, E2 Young-lottery histogram, E3 Rouwenhorst).
They have no reference arithmetic; this module *defines* them for the build, re-using
the reference's conventions wherever one exists:

* income levels exp(y) / mean(exp(y)) (``Aiyagari_Support.py:985``, quirk Q3);
* the EGM step of ``solve_Aiyagari`` (``Aiyagari_Support.py:1423-1520``) with the
  aggregate-M dimension removed: R and w are constants, E = beta * sum(R vP P),
  c = E**(-1/rho), m = a + c, the (1e-7, 1e-7) node prepended (quirk Q4), HARK
  LinearInterp semantics for next-period consumption;
* prices from the Cobb-Douglas firm of ``calc_R_and_W`` (``Aiyagari_Support.py:1886-1890``)
  with L = 1: w(r) = (1-alpha) (alpha/(r+delta))^(alpha/(1-alpha)),
  K_d(r) = (alpha/(r+delta))^(1/(1-alpha)).

Parity for these rows is "oracle-defined" (no reference outputs exist); the Table II
paper values are loose sanity anchors only.
"""
from __future__ import annotations

import numpy as np

from .hark_ks import BORROW_NODE, labor_levels, make_grid_exp_mult, tauchen_for


# --------------------------------------------------------------------------------------
# E3: Rouwenhorst
# --------------------------------------------------------------------------------------
def rouwenhorst(N, rho, sigma_y):
    """Rouwenhorst (1995) / Kopecky-Suen (2010) discretisation of y' = rho y + e with
    unconditional s.d. ``sigma_y`` (the reference's LaborSD is the unconditional s.d.,
    ``Aiyagari_Support.py:885``).  Returns (y[N], P[N, N])."""
    p = (1.0 + rho) / 2.0
    q = p
    P = np.array([[p, 1.0 - p], [1.0 - q, q]])
    for n in range(3, N + 1):
        Z = np.zeros((n, n))
        Z[: n - 1, : n - 1] += p * P
        Z[: n - 1, 1:] += (1.0 - p) * P
        Z[1:, : n - 1] += (1.0 - q) * P
        Z[1:, 1:] += q * P
        Z[1:-1, :] /= 2.0
        P = Z
    if N == 1:
        return np.zeros(1), np.ones((1, 1))
    psi = np.sqrt(N - 1) * sigma_y
    y = np.linspace(-psi, psi, N)
    return y, P


def income_process(n_states, rho, sigma_y, method="tauchen"):
    """(levels, P) for the stationary model.  Tauchen follows the reference exactly
    (``Aiyagari_Support.py:885-887``); Rouwenhorst is E3."""
    if method == "tauchen":
        y, P = tauchen_for(n_states, rho, sigma_y)
    elif method == "rouwenhorst":
        y, P = rouwenhorst(n_states, rho, sigma_y)
    else:
        raise ValueError(method)
    return labor_levels(y), P


def prices(r, alpha, delta):
    """Firm side with L = 1: (w, K_demand)."""
    KtoL = (alpha / (r + delta)) ** (1.0 / (1.0 - alpha))
    w = (1.0 - alpha) * KtoL ** alpha
    return w, KtoL


# --------------------------------------------------------------------------------------
# E1 (inner): stationary EGM
# --------------------------------------------------------------------------------------
def egm_step(m_next, c_next, beta, rho, aGrid, R, w, lab, P, matmul=False):
    """Stationary solve_Aiyagari step.  Tables [S][n_a + 1]; m_next None = terminal c = m.
    matmul=True forms the expectation as one BLAS product V @ P.T (same sums, another
    summation order; used for the large fixtures, tests/golden/make_golden_fullsize.py)."""
    S = P.shape[0]
    nA = aGrid.size
    mN = R * aGrid[:, None] + w * lab[None, :]             # [a, s']
    vP = np.empty((nA, S))
    with np.errstate(all="ignore"):
        for sp in range(S):
            q = mN[:, sp]
            if m_next is None:
                c = q * 1.0
            else:
                x, y = m_next[sp], c_next[sp]
                i = np.maximum(np.searchsorted(x[:-1], q), 1)
                al = (q - x[i - 1]) / (x[i] - x[i - 1])
                c = (1.0 - al) * y[i - 1] + al * y[i]
                c[q < x[0]] = np.nan
            vP[:, sp] = c ** -rho
        V = R * vP
        E = beta * (V @ P.T if matmul else np.sum(V[:, None, :] * P[None, :, :], axis=2))
        cNow = E ** (-1.0 / rho)
    mNow = aGrid[:, None] + cNow
    m_out = np.empty((S, nA + 1))
    c_out = np.empty((S, nA + 1))
    m_out[:, 0] = BORROW_NODE
    c_out[:, 0] = BORROW_NODE
    m_out[:, 1:] = mNow.T
    c_out[:, 1:] = cNow.T
    return m_out, c_out


def egm_solve(beta, rho, aGrid, R, w, lab, P, tol=1e-6, max_cycles=5000, matmul=False):
    """HARK-style infinite-horizon loop (cold start, sup-norm over m and c, stop when
    dist <= tol)."""
    m, c = egm_step(None, None, beta, rho, aGrid, R, w, lab, P, matmul)
    cycles = 1
    while True:
        m2, c2 = egm_step(m, c, beta, rho, aGrid, R, w, lab, P, matmul)
        with np.errstate(invalid="ignore"):
            dist = max(np.max(np.abs(m2 - m)), np.max(np.abs(c2 - c)))
        go = dist > tol and cycles < max_cycles
        m, c = m2, c2
        cycles += 1
        if not go:
            return m, c, cycles, dist


# --------------------------------------------------------------------------------------
# E2: Young-lottery histogram
# --------------------------------------------------------------------------------------
def savings_lottery(m_tab, c_tab, aGrid, R, w, lab):
    """For every (s, j): a' = m - c_s(m), m = R a_j + w l_s, and its lottery onto aGrid:
    (lo index, weight on lo).  a' <= a_0 -> (0, 1); a' >= a_last -> (n-2, 0)."""
    S = m_tab.shape[0]
    nA = aGrid.size
    lo = np.empty((S, nA), dtype=np.int64)
    wlo = np.empty((S, nA))
    ap = np.empty((S, nA))
    for s in range(S):
        q = R * aGrid + w * lab[s]
        x, y = m_tab[s], c_tab[s]
        i = np.maximum(np.searchsorted(x[:-1], q), 1)
        al = (q - x[i - 1]) / (x[i] - x[i - 1])
        c = (1.0 - al) * y[i - 1] + al * y[i]
        a1 = q - c
        ap[s] = a1
        j = np.searchsorted(aGrid, a1, side="right") - 1
        j = np.clip(j, 0, nA - 2)
        wl = (aGrid[j + 1] - a1) / (aGrid[j + 1] - aGrid[j])
        wl = np.clip(wl, 0.0, 1.0)
        lo[s] = j
        wlo[s] = wl
    return lo, wlo, ap


def hist_step(mass, lo, wlo, P):
    """mass'[s', .] = sum_s P[s, s'] T_s, T_s = lottery push of mass[s, .]."""
    S, nA = mass.shape
    T = np.zeros((S, nA))
    for s in range(S):
        np.add.at(T[s], lo[s], wlo[s] * mass[s])
        np.add.at(T[s], lo[s] + 1, (1.0 - wlo[s]) * mass[s])
    return P.T @ T


def hist_step_fast(mass, lo, wlo, P):
    """hist_step with np.bincount in place of np.add.at (the vectorised-NumPy CPU bound
    bench.py times; same sums, summation order of equal destinations may differ)."""
    S, nA = mass.shape
    rows = (np.arange(S)[:, None] * nA + lo).ravel()
    a = (wlo * mass).ravel()
    b = ((1.0 - wlo) * mass).ravel()
    T = np.bincount(rows, weights=a, minlength=S * nA) + np.bincount(rows + 1, weights=b, minlength=S * nA + 1)[:S * nA]
    return P.T @ T.reshape(S, nA)


def stationary_hist(lo, wlo, P, nA, tol=1e-12, max_iter=100000, mass0=None, step=None):
    S = P.shape[0]
    step = hist_step if step is None else step
    mass = np.full((S, nA), 1.0 / (S * nA)) if mass0 is None else mass0.copy()
    for it in range(1, max_iter + 1):
        new = step(mass, lo, wlo, P)
        d = np.max(np.abs(new - mass))
        mass = new
        if d < tol:
            return mass, it, d
    return mass, max_iter, d


# --------------------------------------------------------------------------------------
# E1 (outer): GE bisection on r
# --------------------------------------------------------------------------------------
def capital_supply(r, cal, aGrid, lab, P, egm_tol=1e-8, hist_tol=1e-12, fast=False, egm_matmul=False):
    w, _ = prices(r, cal["CapShare"], cal["DeprFac"])
    R = 1.0 + r
    m, c, cycles, _ = egm_solve(cal["DiscFac"], cal["CRRA"], aGrid, R, w, lab, P, tol=egm_tol, matmul=egm_matmul)
    lo, wlo, _ = savings_lottery(m, c, aGrid, R, w, lab)
    mass, iters, _ = stationary_hist(lo, wlo, P, aGrid.size, tol=hist_tol, step=hist_step_fast if fast else None)
    K = float(np.sum(mass * aGrid[None, :]))
    return K, dict(m=m, c=c, mass=mass, cycles=cycles, hist_iters=iters)


def ge_bisect(cal, aGrid, lab, P, r_lo=None, r_hi=None, r_tol=1e-7, max_iter=60, **kw):
    """Bisection on r for K_s(r) = K_d(r).  Returns dict(r, K, KtoY, saving_rate, iters,
    lo, hi) -- (lo, hi) the final bracket, r its midpoint."""
    a, d, b = cal["CapShare"], cal["DeprFac"], cal["DiscFac"]
    lo = -d * 0.5 if r_lo is None else r_lo
    hi = 1.0 / b - 1.0 - 1e-9 if r_hi is None else r_hi
    it = 0
    while hi - lo > r_tol and it < max_iter:
        mid = 0.5 * (lo + hi)
        Ks, _ = capital_supply(mid, cal, aGrid, lab, P, **kw)
        _, Kd = prices(mid, a, d)
        if Ks > Kd:
            hi = mid
        else:
            lo = mid
        it += 1
    r = 0.5 * (lo + hi)
    _, K = prices(r, a, d)
    KtoY = K ** (1.0 - a)
    return dict(r=r, K=K, KtoY=KtoY, saving_rate=d * KtoY, iters=it, lo=lo, hi=hi)


def make_stationary_grid(aMin=0.001, aMax=50.0, aCount=32, aNestFac=2):
    return make_grid_exp_mult(aMin, aMax, aCount, aNestFac)
