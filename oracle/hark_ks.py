"""CPU ORACLE (test infrastructure only) -- Krusell-Smith-form Aiyagari block.

NumPy restatement of the reference's hot path, ``/root/reference/Aiyagari_Support.py``
(cited as ``AS:<line>``) and ``Aiyagari-HARK.py`` (``AH:<line>``), together with the
econ-ark **HARK 0.12** library routines it calls (``[HARK]``; the library is pinned
at ``requirements.txt:1`` and is *not* present in the reference or in this image, so
its published 0.12 algorithm is restated here: SURVEY.md §8a rows A1, A2, A9-A12,
B6, C3, C5).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module.  Two granularities are provided:

* ``*_ref`` functions follow the reference literally, including its 4-D tiled
  ``[a, M, s, s']`` arrays (28x redundant over ``s``) and HARK's per-state interpolant
  objects.  Use them at reference sizes (N_a = 32).
* the unsuffixed vectorised versions compute exactly the same floating-point
  operations element by element, without the redundant ``s`` axis, so they can run
  at N_a = 10 000.  ``tests/test_oracle.py`` checks the two are bit-identical.

Parity: "partially pinned" -- see oracle/__init__.py and DESIGN.md.
"""
from __future__ import annotations

import math
from copy import deepcopy

import numpy as np
from scipy import stats

# --------------------------------------------------------------------------------------
# Calibration dictionaries (AS:752-755 agents, AS:1525-1551 economy)
# --------------------------------------------------------------------------------------
MGRID_BASE = np.array([0.1, 0.3, 0.6, 0.8, 0.9, 0.95, 0.98, 1.0, 1.02, 1.05, 1.1, 1.2, 1.6, 2.0, 3.0])

INIT_AGENTS = dict(LaborStatesNo=7, LaborAR=0.6, LaborSD=0.2, T_cycle=1, DiscFac=0.96, CRRA=1.0,
                   LbrInd=1.0, aMin=0.001, aMax=50.0, aCount=32, aNestFac=2,
                   MgridBase=MGRID_BASE.copy(), AgentCount=140)

INIT_ECONOMY = {
    "verbose": True, "LaborStatesNo": 7, "LaborAR": 0.6, "LaborSD": 0.2, "act_T": 11000,
    "T_discard": 1000, "DampingFac": 0.5, "intercept_prev": [0.0, 0.0], "slope_prev": [1.0, 1.0],
    "DiscFac": 0.96, "CRRA": 1.0, "LbrInd": 1.0, "ProdB": 1.0, "ProdG": 1.0, "CapShare": 0.36,
    "DeprFac": 0.08, "DurMeanB": 8.0, "DurMeanG": 8.0, "SpellMeanB": 2.5, "SpellMeanG": 1.5,
    "UrateB": 0.0, "UrateG": 0.0, "RelProbBG": 0.75, "RelProbGB": 1.25, "MrkvNow_init": 0,
}

AGENT_TOLERANCE = 1e-6      # [HARK] AgentType default tolerance (not overridden, AS:752-755)
MAX_CYCLES = 5000           # [HARK] solve_agent escape clause
MARKET_TOLERANCE = 0.01     # AS:1574
MAX_LOOPS = 1000            # [HARK] Market.max_loops
BORROW_NODE = 0.0000001     # AS:1503-1504


# --------------------------------------------------------------------------------------
# [HARK] utilities / distribution (rows A1, A2)
# --------------------------------------------------------------------------------------
def make_grid_exp_mult(ming, maxg, ng, timestonest=20):
    """[HARK 0.12] utilities.make_grid_exp_mult, called at AS:880."""
    if timestonest > 0:
        Lming = ming
        Lmaxg = maxg
        for _ in range(timestonest):
            Lming = np.log(Lming + 1)
            Lmaxg = np.log(Lmaxg + 1)
        grid = np.linspace(Lming, Lmaxg, ng)
        for _ in range(timestonest):
            grid = np.exp(grid) - 1
    else:
        Lming = np.log(ming)
        Lmaxg = np.log(maxg)
        Lstep = (Lmaxg - Lming) / (ng - 1)
        grid = np.exp(np.arange(Lming, Lmaxg + 0.000001, Lstep))
    return grid


def make_tauchen_ar1(N, sigma=1.0, ar_1=0.9, bound=3.0):
    """[HARK 0.12] distribution.make_tauchen_ar1, called at AS:887 and AS:1696."""
    yN = bound * sigma / ((1 - ar_1 ** 2) ** 0.5)
    y = np.linspace(-yN, yN, N)
    d = y[1] - y[0]
    trans = np.ones((N, N))
    for j in range(N):
        for k_1 in range(N - 2):
            k = k_1 + 1
            trans[j, k] = (stats.norm.cdf((y[k] + d / 2.0 - ar_1 * y[j]) / sigma)
                           - stats.norm.cdf((y[k] - d / 2.0 - ar_1 * y[j]) / sigma))
        trans[j, 0] = stats.norm.cdf((y[0] + d / 2.0 - ar_1 * y[j]) / sigma)
        trans[j, N - 1] = 1.0 - stats.norm.cdf((y[N - 1] - d / 2.0 - ar_1 * y[j]) / sigma)
    return y, trans


def tauchen_for(LaborStatesNo, LaborAR, LaborSD):
    """AS:885-887 / AS:1694-1696: sigma = LaborSD * sqrt(1 - rho^2), bound 3."""
    SDshock = LaborSD * (1 - (LaborAR ** 2)) ** (0.5)
    return make_tauchen_ar1(LaborStatesNo, sigma=SDshock, ar_1=LaborAR, bound=3.0)


def labor_levels(tauchen_y):
    """AS:985 / AS:1265: exp(y) normalised by its simple mean (quirk Q3)."""
    return np.exp(tauchen_y) / np.mean(np.exp(tauchen_y))


def CRRAutilityP(c, gam):
    """[HARK] utilities.CRRAutilityP (AS:22)."""
    return c ** -gam


# --------------------------------------------------------------------------------------
# [HARK] interpolation (rows A9-A11)
# --------------------------------------------------------------------------------------
class LinearInterp:
    """[HARK 0.12] LinearInterp(x, y) with lower_extrap=False (built at AS:1512).

    i = max(searchsorted(x[:-1], q, 'left'), 1); linear extrapolation above the grid;
    NaN below x[0]."""

    distance_criteria = ["x_list", "y_list"]

    def __init__(self, x_list, y_list):
        self.x_list = np.array(x_list, dtype=np.float64).flatten()
        self.y_list = np.array(y_list, dtype=np.float64).flatten()
        self.x_n = self.x_list.size

    def _evaluate(self, x):
        i = np.maximum(np.searchsorted(self.x_list[:-1], x), 1)
        alpha = (x - self.x_list[i - 1]) / (self.x_list[i] - self.x_list[i - 1])
        y = (1.0 - alpha) * self.y_list[i - 1] + alpha * self.y_list[i]
        y[x < self.x_list[0]] = np.nan
        return y

    def __call__(self, x):
        z = np.asarray(x, dtype=np.float64)
        return self._evaluate(z.flatten()).reshape(z.shape)


class LinearInterpOnInterp1D:
    """[HARK 0.12] LinearInterpOnInterp1D(xInterpolators, y_values) (built at AS:1513).

    Vector path: y_pos = clip(searchsorted(y_list, y, 'left'), 1, y_n - 1);
    f = (1 - alpha) f_{k-1}(x) + alpha f_k(x); linear extrapolation in y."""

    distance_criteria = ["xInterpolators", "y_list"]

    def __init__(self, xInterpolators, y_values):
        self.xInterpolators = xInterpolators
        self.y_list = np.asarray(y_values, dtype=np.float64)
        self.y_n = self.y_list.size

    def _evaluate(self, x, y):
        m = len(x)
        y_pos = np.searchsorted(self.y_list, y)
        y_pos[y_pos > self.y_n - 1] = self.y_n - 1
        y_pos[y_pos < 1] = 1
        f = np.zeros(m) + np.nan
        if y.size > 0:
            for i in range(1, self.y_n):
                c = y_pos == i
                if np.any(c):
                    alpha = (y[c] - self.y_list[i - 1]) / (self.y_list[i] - self.y_list[i - 1])
                    f[c] = (1 - alpha) * self.xInterpolators[i - 1](x[c]) + alpha * self.xInterpolators[i](x[c])
        return f

    def __call__(self, x, y):
        xa = np.asarray(x, dtype=np.float64)
        ya = np.asarray(y, dtype=np.float64)
        return self._evaluate(xa.flatten(), ya.flatten()).reshape(xa.shape)


class IdentityFunction:
    """[HARK] IdentityFunction(n_dims=2): returns its first argument (AS:898)."""

    distance_criteria = ["i_dim"]

    def __init__(self, i_dim=0, n_dims=1):
        self.i_dim = i_dim
        self.n_dims = n_dims

    def __call__(self, *args):
        return np.asarray(args[self.i_dim], dtype=np.float64) * 1.0


class MargValueFuncCRRA:
    """[HARK] MargValueFuncCRRA(cFunc, CRRA): vP = cFunc(...)**-CRRA (AS:899-900, AS:1514)."""

    distance_criteria = ["cFunc", "CRRA"]

    def __init__(self, cFunc, CRRA):
        self.cFunc = cFunc
        self.CRRA = CRRA

    def __call__(self, *args):
        return CRRAutilityP(self.cFunc(*args), gam=self.CRRA)


class ConsumerSolution:
    distance_criteria = ["vPfunc"]

    def __init__(self, cFunc=None, vPfunc=None):
        self.cFunc = cFunc
        self.vPfunc = vPfunc


def distance_metric(A, B):
    """[HARK 0.12] core.distance_metric / MetricObject.distance restated."""
    if isinstance(A, list) and isinstance(B, list):
        if len(A) == len(B):
            return max(distance_metric(a, b) for a, b in zip(A, B))
        return float(abs(len(A) - len(B)))
    if isinstance(A, (int, float)) and isinstance(B, (int, float)):
        return float(abs(A - B))
    if hasattr(A, "shape") and hasattr(B, "shape"):
        if A.shape == B.shape:
            return np.max(abs(A - B))
        return np.max(abs(A.flatten().shape[0] - B.flatten().shape[0]))
    if type(A).__name__ == type(B).__name__:
        dist = [0.0]
        for attr in A.distance_criteria:
            try:
                dist.append(distance_metric(getattr(A, attr), getattr(B, attr)))
            except AttributeError:
                dist.append(1000.0)
        return max(dist)
    return 1000.0


# --------------------------------------------------------------------------------------
# Economy setup (rows A4, A5)
# --------------------------------------------------------------------------------------
def steady_state(p):
    """AiyagariEconomy.update closed forms (AS:1606-1615)."""
    KtoLSS = ((1.0 ** p["CRRA"] / p["DiscFac"] - (1.0 - p["DeprFac"])) / p["CapShare"]) ** (1.0 / (p["CapShare"] - 1.0))
    KSS = KtoLSS * p["LbrInd"]
    WSS = (1.0 - p["CapShare"]) * KtoLSS ** (p["CapShare"])
    RSS = 1.0 + p["CapShare"] * KtoLSS ** (p["CapShare"] - 1.0) - p["DeprFac"]
    MSS = KSS * RSS + WSS * p["LbrInd"]
    return dict(KtoLSS=KtoLSS, KSS=KSS, WSS=WSS, RSS=RSS, MSS=MSS, KtoYSS=KtoLSS ** (1.0 - p["CapShare"]))


def make_MrkvArray(p):
    """AiyagariEconomy.make_MrkvArray (AS:1639-1791), generalised over LaborStatesNo.

    The reference writes the 49 blocks of kron(P_tauchen, MrkvEmplArray) by hand
    (AS:1715-1780); here each block is formed the same way (elementwise product of
    MrkvEmplArray with one Tauchen entry) and concatenated in the same order."""
    ProbBG = 1.0 / p["DurMeanB"]
    ProbGB = 1.0 / p["DurMeanG"]
    ProbBB = 1.0 - ProbBG
    ProbGG = 1.0 - ProbGB
    MrkvAggArray = np.array([[ProbBB, ProbBG], [ProbGB, ProbGG]])
    E = np.zeros((4, 4))
    UB, UG = p["UrateB"], p["UrateG"]
    E[0, 1] = ProbBB * 1.0 / p["SpellMeanB"]
    E[0, 0] = ProbBB * (1 - 1.0 / p["SpellMeanB"])
    E[1, 0] = UB / (1.0 - UB) * E[0, 1]
    E[1, 1] = ProbBB - E[1, 0]
    E[2, 3] = ProbGG * 1.0 / p["SpellMeanG"]
    E[2, 2] = ProbGG * (1 - 1.0 / p["SpellMeanG"])
    E[3, 2] = UG / (1.0 - UG) * E[2, 3]
    E[3, 3] = ProbGG - E[3, 2]
    E[0, 2] = p["RelProbBG"] * E[2, 2] / ProbGG * ProbBG
    E[0, 3] = ProbBG - E[0, 2]
    E[1, 2] = (ProbBG * UG - UB * E[0, 2]) / (1.0 - UB)
    E[1, 3] = ProbBG - E[1, 2]
    E[2, 0] = p["RelProbGB"] * E[0, 0] / ProbBB * ProbGB
    E[2, 1] = ProbGB - E[2, 0]
    E[3, 0] = (ProbGB * UB - UG * E[2, 0]) / (1.0 - UG)
    E[3, 1] = ProbGB - E[3, 0]
    T = tauchen_for(p["LaborStatesNo"], p["LaborAR"], p["LaborSD"])
    n = p["LaborStatesNo"]
    rows = []
    for i in range(n):
        blocks = [np.array([element * T[1][i, j] for element in E]) for j in range(n)]
        rows.append(np.concatenate(blocks, axis=1))
    MrkvIndArray = np.concatenate(rows, axis=0)
    assert np.all(MrkvIndArray >= 0.0), "Invalid idiosyncratic transition probabilities!"
    return dict(MrkvArray=MrkvAggArray, MrkvIndArray=MrkvIndArray, MrkvEmplArray=E, TauchenAux=T)


def make_Mrkv_history(MrkvArray, act_T, MrkvNow_init=0, seed=0):
    """AS:1793-1805 with [HARK 0.12] MarkovProcess(seed=0).draw -> RNG.choice(n, p=row)."""
    rng = np.random.RandomState(seed)
    hist = np.zeros(act_T, dtype=int)
    now = MrkvNow_init
    for s in range(act_T):
        hist[s] = now
        now = rng.choice(MrkvArray.shape[1], p=MrkvArray[now, :])
    return hist


class AggregateSavingRule:
    """AS:1973-2005."""

    distance_criteria = ["slope", "intercept"]

    def __init__(self, intercept, slope):
        self.intercept = intercept
        self.slope = slope

    def __call__(self, Mnow):
        return np.exp(self.intercept + self.slope * np.log(Mnow))


class AggShocksDynamicRule:
    """AS:2008-2020."""

    distance_criteria = ["AFunc"]

    def __init__(self, AFunc):
        self.AFunc = AFunc


# --------------------------------------------------------------------------------------
# precompute_arrays (row A7)
# --------------------------------------------------------------------------------------
def _agg_state_of(sp):
    """Aggregate state g(s') = (s' mod 4) div 2 (AS:927: KnextB, KnextB, KnextG, KnextG ...)."""
    return (np.asarray(sp) % 4) // 2


def next_prices(AFunc, Mgrid, n_lab, e):
    """Per-(M, s') next-period R, W, M' exactly as AS:923-976 computes them elementwise.

    Returns Rnext[k, s'], Wnext[k, s'], Mnext[k, s'] (each float64 [n_M, 4 n_lab])."""
    S = 4 * n_lab
    g = _agg_state_of(np.arange(S))
    AnowB = AFunc[0](Mgrid)
    AnowG = AFunc[1](Mgrid)
    Knext = np.where(g[None, :] == 0, AnowB[:, None], AnowG[:, None])
    Lnext = np.where(g == 0, (1.0 - e["UrateB"]) * e["LbrInd"], (1.0 - e["UrateG"]) * e["LbrInd"])[None, :] * np.ones_like(Knext)
    Znext = np.where(g == 0, e["ProdB"], e["ProdG"])[None, :] * np.ones_like(Knext)
    KtoLnext = Knext / Lnext
    Rnext = 1.0 + Znext * e["CapShare"] * KtoLnext ** (e["CapShare"] - 1.0) - e["DeprFac"]
    Wnext = Znext * (1.0 - e["CapShare"]) * KtoLnext ** e["CapShare"]
    Ynext = Znext * Knext ** e["CapShare"] * Lnext ** (1.0 - e["CapShare"])
    Mnext = (1.0 - e["DeprFac"]) * Knext + Ynext
    return Rnext, Wnext, Mnext


def precompute_arrays_ref(aGrid, Mgrid, AFunc, LSStates, MrkvIndArray, e):
    """AiyagariType.precompute_arrays (AS:906-1037), literal 4-D [a, M, s, s'] layout."""
    aCount, Mcount, S = aGrid.size, Mgrid.size, MrkvIndArray.shape[0]
    n_lab = S // 4
    Rk, Wk, Mk = next_prices(AFunc, Mgrid, n_lab, e)
    aNow_tiled = np.tile(np.reshape(aGrid, [aCount, 1, 1, 1]), [1, Mcount, S, S])
    Rnext_tiled = np.tile(Rk[None, :, None, :], [aCount, 1, S, 1])
    Wnext_tiled = np.tile(Wk[None, :, None, :], [aCount, 1, S, 1])
    Mnext_tiled = np.tile(Mk[None, :, None, :], [aCount, 1, S, 1])
    lNext_tiled = np.zeros([aCount, Mcount, S, S])
    for sp in range(S):
        lNext_tiled[:, :, :, sp] = LSStates[sp // 4]          # AS:990-1018 (quirk Q2)
    mNext = Rnext_tiled * aNow_tiled + Wnext_tiled * lNext_tiled   # AS:1024
    Probs_tiled = np.tile(np.reshape(MrkvIndArray, [1, 1, S, S]), [aCount, Mcount, 1, 1])
    return dict(ProbArray=Probs_tiled, mNextArray=mNext, MnextArray=Mnext_tiled, RnextArray=Rnext_tiled)


# --------------------------------------------------------------------------------------
# solve_Aiyagari (row A8), literal form
# --------------------------------------------------------------------------------------
def terminal_solution(S, CRRA):
    """update_solution_terminal (AS:892-904): c = m, vP = m**-CRRA."""
    cF = S * [IdentityFunction(n_dims=2)]
    return ConsumerSolution(cFunc=cF, vPfunc=[MargValueFuncCRRA(cF[j], CRRA) for j in range(S)])


def solve_Aiyagari_ref(solution_next, DiscFac, CRRA, aGrid, Mgrid, mNextArray, MnextArray,
                       ProbArray, RnextArray, LaborStatesNo):
    """solve_Aiyagari (AS:1423-1520), literal."""
    n = LaborStatesNo
    vPnext = np.zeros_like(mNextArray)
    for j in range(4 * n):
        vPnext[:, :, :, j] = solution_next.vPfunc[j](mNextArray[:, :, :, j], MnextArray[:, :, :, j])
    EndOfPrdvP = DiscFac * np.sum(RnextArray * vPnext * ProbArray, axis=3)
    cNow = EndOfPrdvP ** (-1.0 / CRRA)
    aCount, Mcount = aGrid.size, Mgrid.size
    aNow = np.tile(np.reshape(aGrid, [aCount, 1, 1]), [1, Mcount, 4 * n])
    mNow = aNow + cNow
    cNow = np.concatenate([(np.zeros([1, Mcount, 4 * n]) + BORROW_NODE), cNow], axis=0)
    mNow = np.concatenate([(np.zeros([1, Mcount, 4 * n]) + BORROW_NODE), mNow], axis=0)
    cFunc_by_state, vPfunc_by_state = [], []
    for j in range(4 * n):
        cFunc_by_M = [LinearInterp(mNow[:, k, j], cNow[:, k, j]) for k in range(Mcount)]
        cFunc_j = LinearInterpOnInterp1D(cFunc_by_M, Mgrid)
        cFunc_by_state.append(cFunc_j)
        vPfunc_by_state.append(MargValueFuncCRRA(cFunc_j, CRRA))
    return ConsumerSolution(cFunc=cFunc_by_state, vPfunc=vPfunc_by_state)


def solution_to_tables(sol):
    """Stack a solve_Aiyagari ConsumerSolution into (m, c) tables [S][n_M][n_a + 1]."""
    m = np.array([[xi.x_list for xi in cf.xInterpolators] for cf in sol.cFunc])
    c = np.array([[xi.y_list for xi in cf.xInterpolators] for cf in sol.cFunc])
    return m, c


def solve_agent_ref(DiscFac, CRRA, aGrid, Mgrid, arrays, LaborStatesNo, tol=AGENT_TOLERANCE,
                    max_cycles=MAX_CYCLES):
    """[HARK 0.12] solve_agent, infinite horizon (cycles = 0, AH:237), cold start (Q12)."""
    S = 4 * LaborStatesNo
    solution_last = terminal_solution(S, CRRA)
    completed = 0
    go = True
    dist = 100.0
    with np.errstate(all="ignore"):
        while go:
            now = solve_Aiyagari_ref(solution_last, DiscFac, CRRA, aGrid, Mgrid, arrays["mNextArray"],
                                     arrays["MnextArray"], arrays["ProbArray"], arrays["RnextArray"],
                                     LaborStatesNo)
            if completed > 0:
                dist = distance_metric(now, solution_last)
                go = dist > tol and completed < max_cycles
            solution_last = now
            completed += 1
    return solution_last, completed, dist


# --------------------------------------------------------------------------------------
# Vectorised (bit-identical) EGM for larger grids
# --------------------------------------------------------------------------------------
def _interp_rows(xr, yr, q):
    """HARK LinearInterp on many rows at once: xr, yr [R, n]; q [R, Q] -> [R, Q].

    Per row identical to LinearInterp._evaluate (searchsorted(x[:-1], q, 'left'))."""
    R, n = xr.shape
    out = np.empty(q.shape)
    for r in range(R):
        x, y, qq = xr[r], yr[r], q[r]
        i = np.maximum(np.searchsorted(x[:-1], qq), 1)
        alpha = (qq - x[i - 1]) / (x[i] - x[i - 1])
        v = (1.0 - alpha) * y[i - 1] + alpha * y[i]
        v[qq < x[0]] = np.nan
        out[r] = v
    return out


def eval_policy_2d(m_tab, c_tab, Mgrid, s, mq, Mq):
    """cFunc_s(mq, Mq) for policy tables [S][n_M][n_a+1], HARK LinearInterpOnInterp1D
    semantics for a scalar ``Mq`` shared by all queries ``mq`` (1-D array)."""
    n_M = Mgrid.size
    k = int(np.searchsorted(Mgrid, Mq))
    k = min(max(k, 1), n_M - 1)
    alpha = (Mq - Mgrid[k - 1]) / (Mgrid[k] - Mgrid[k - 1])
    lo = _interp_rows(m_tab[s, k - 1][None], c_tab[s, k - 1][None], np.asarray(mq)[None])[0]
    hi = _interp_rows(m_tab[s, k][None], c_tab[s, k][None], np.asarray(mq)[None])[0]
    return (1 - alpha) * lo + alpha * hi


def egm_step(m_next, c_next, DiscFac, CRRA, aGrid, Mgrid, Rk, Wk, Mk, LSStates, P):
    """One solve_Aiyagari step on tables; bit-identical to solve_Aiyagari_ref.

    m_next/c_next: [S][n_M][n_a+1] or None for the terminal IdentityFunction guess.
    Rk/Wk/Mk: [n_M, S] next-period R, W, M' (next_prices)."""
    S = P.shape[0]
    nA, nM = aGrid.size, Mgrid.size
    lab = np.array([LSStates[sp // 4] for sp in range(S)])
    # mNext[a, k, s'] = R a + W l (AS:1024), independent of the current state s
    mN = Rk[None, :, :] * aGrid[:, None, None] + Wk[None, :, :] * lab[None, None, :]
    vP = np.empty((nA, nM, S))
    with np.errstate(all="ignore"):
        for sp in range(S):
            if m_next is None:
                c = mN[:, :, sp] * 1.0
            else:
                # LinearInterpOnInterp1D in M at M' = Mk[k, sp] (constant over a)
                c = np.empty((nA, nM))
                y_list = Mgrid
                y_pos = np.searchsorted(y_list, Mk[:, sp])
                y_pos[y_pos > nM - 1] = nM - 1
                y_pos[y_pos < 1] = 1
                for k in range(nM):
                    i = y_pos[k]
                    alpha = (Mk[k, sp] - y_list[i - 1]) / (y_list[i] - y_list[i - 1])
                    q = mN[:, k, sp]
                    f0 = _interp_rows(m_next[sp, i - 1][None], c_next[sp, i - 1][None], q[None])[0]
                    f1 = _interp_rows(m_next[sp, i][None], c_next[sp, i][None], q[None])[0]
                    c[:, k] = (1 - alpha) * f0 + alpha * f1
            vP[:, :, sp] = c ** -CRRA
        # np.sum(R * vP * P, axis=3): same elementwise products, same pairwise reduction
        V = Rk[None, :, :] * vP                               # [a, k, s']
        E = np.empty((nA, nM, S))
        chunk = max(1, 200000 // (nM * S * S))
        for a0 in range(0, nA, chunk):
            a1 = min(nA, a0 + chunk)
            E[a0:a1] = DiscFac * np.sum(V[a0:a1, :, None, :] * P[None, None, :, :], axis=3)
        cNow = E ** (-1.0 / CRRA)
    mNow = aGrid[:, None, None] + cNow
    m_out = np.empty((S, nM, nA + 1))
    c_out = np.empty((S, nM, nA + 1))
    m_out[:, :, 0] = BORROW_NODE
    c_out[:, :, 0] = BORROW_NODE
    m_out[:, :, 1:] = np.transpose(mNow, (2, 1, 0))
    c_out[:, :, 1:] = np.transpose(cNow, (2, 1, 0))
    return m_out, c_out


def egm_solve(DiscFac, CRRA, aGrid, Mgrid, Rk, Wk, Mk, LSStates, P, tol=AGENT_TOLERANCE,
              max_cycles=MAX_CYCLES):
    """[HARK 0.12] solve_agent loop on tables (cold start).  Returns (m, c, cycles, dist)."""
    m, c = egm_step(None, None, DiscFac, CRRA, aGrid, Mgrid, Rk, Wk, Mk, LSStates, P)
    completed = 1
    dist = 100.0
    while True:
        m2, c2 = egm_step(m, c, DiscFac, CRRA, aGrid, Mgrid, Rk, Wk, Mk, LSStates, P)
        with np.errstate(invalid="ignore"):
            dist = max(np.max(np.abs(m2 - m)), np.max(np.abs(c2 - c)))
        go = dist > tol and completed < max_cycles
        m, c = m2, c2
        completed += 1
        if not go:
            break
    return m, c, completed, dist


# --------------------------------------------------------------------------------------
# Panel simulation (rows B1-B6)
# --------------------------------------------------------------------------------------
def sim_birth_labor(AgentCount, LaborStatesNo, UrateB, seed=0, Mrkv=0, UrateG=None, return_rng=False):
    """initialize_sim / sim_birth (AS:1164-1214) with [HARK] reset_rng (RandomState(seed)).

    Returns (EmpNow bool[N], LaborSupplyState int[N]) -- and the agent RNG, which the
    per-period employment permutations continue (AS:1239-1240), if return_rng.  Two
    RNG.permutation calls, in the reference's order (AS:1212, AS:1214); the unemployment
    count is the birth period's state's (AS:1185-1190)."""
    rng = np.random.RandomState(seed)
    N = AgentCount
    if Mrkv == 0:
        unemp_N = int(np.round(UrateB * N))
    elif Mrkv == 1:
        unemp_N = int(np.round((UrateB if UrateG is None else UrateG) * N))
    else:
        raise ValueError("Illegal macroeconomic state: MrkvNow must be 0 or 1")
    emp_N = AgentCount - unemp_N
    EmpNew = np.concatenate([np.zeros(unemp_N, dtype=bool), np.ones(emp_N, dtype=bool)])
    LSNew = np.empty(0)
    for n in range(LaborStatesNo):
        LSNew = np.concatenate((LSNew, n * np.ones(int(AgentCount / LaborStatesNo))), axis=0)
    LSNew2 = np.array([int(el) for el in LSNew])
    emp = rng.permutation(EmpNew)
    lab = rng.permutation(LSNew2)
    if return_rng:
        return emp, lab, rng
    return emp, lab


def make_emp_idx_arrays(AgentCount, UrateB, UrateG, MrkvEmplArray, MrkvAggArray):
    """AiyagariType.make_emp_idx_arrays (AS:1042-1156): emp_permute[j][k] / unemp_permute[j][k]
    are the boolean arrays whose random permutations give, for the macro transition j -> k,
    this period's employment of last period's employed / unemployed agents (exact counts).
    Written out per transition as the reference does (same products, same rounding)."""
    E, A = MrkvEmplArray, MrkvAggArray
    B_unemp_N = int(np.round(UrateB * AgentCount))
    B_emp_N = AgentCount - B_unemp_N
    G_unemp_N = int(np.round(UrateG * AgentCount))
    G_emp_N = AgentCount - G_unemp_N

    def pair(stay_emp, become_unemp, become_emp, stay_unemp):
        unemp_p = np.concatenate([np.ones(become_emp, dtype=bool), np.zeros(stay_unemp, dtype=bool)])
        emp_p = np.concatenate([np.ones(stay_emp, dtype=bool), np.zeros(become_unemp, dtype=bool)])
        return emp_p, unemp_p

    BB_stay_unemp_N = int(np.round(B_unemp_N * E[0, 0] / A[0, 0]))
    BB_stay_emp_N = int(np.round(B_emp_N * (E[1, 1]) / A[0, 0]))
    BB = pair(BB_stay_emp_N, B_unemp_N - BB_stay_unemp_N, B_emp_N - BB_stay_emp_N, BB_stay_unemp_N)
    BG_stay_unemp_N = int(np.round(B_unemp_N * E[0, 2] / A[0, 1]))
    BG_stay_emp_N = int(np.round(B_emp_N * (E[1, 3]) / A[0, 1]))
    BG = pair(BG_stay_emp_N, G_unemp_N - BG_stay_unemp_N, G_emp_N - BG_stay_emp_N, BG_stay_unemp_N)
    GB_stay_unemp_N = int(np.round(G_unemp_N * E[2, 0] / A[1, 0]))
    GB_stay_emp_N = int(np.round(G_emp_N * E[3, 1] / A[1, 0]))
    GB = pair(GB_stay_emp_N, B_unemp_N - GB_stay_unemp_N, B_emp_N - GB_stay_emp_N, GB_stay_unemp_N)
    GG_stay_unemp_N = int(np.round(G_unemp_N * E[2, 2] / A[1, 1]))
    GG_stay_emp_N = int(np.round(G_emp_N * E[3, 3] / A[1, 1]))
    GG = pair(GG_stay_emp_N, G_unemp_N - GG_stay_unemp_N, G_emp_N - GG_stay_emp_N, GG_stay_unemp_N)
    return dict(emp=[[BB[0], BG[0]], [GB[0], GG[0]]], unemp=[[BB[1], BG[1]], [GB[1], GG[1]]])


def employment_step(emp_prev, mrkv_now, UrateB, perms, rng):
    """get_shocks employment part (AS:1222-1240): the previous macro state is read off
    last period's unemployment rate (AS:1227, a float comparison with UrateB), then the
    employed and the unemployed are each given a permutation of their transition array
    (agent RNG, employed first).  Raises like NumPy's boolean assignment does when an
    array's length differs from the group it is assigned to."""
    employed = np.asarray(emp_prev).astype(bool)
    unemployed = np.logical_not(employed)
    mrkv_prev = int((unemployed.sum() / float(employed.size)) != UrateB)
    emp_p = perms["emp"][mrkv_prev][int(mrkv_now)]
    unemp_p = perms["unemp"][mrkv_prev][int(mrkv_now)]
    EmpNow = np.empty(employed.size)
    EmpNow[employed] = rng.permutation(emp_p)
    EmpNow[unemployed] = rng.permutation(unemp_p)
    return EmpNow.astype(bool)


def choice_cdf(P_row):
    """np.random.choice(p=row) inverse-CDF table (NumPy legacy RandomState.choice)."""
    cdf = np.asarray(P_row, dtype=np.float64).cumsum()
    cdf /= cdf[-1]
    return cdf


def draw_labor(lab_prev, u, cdf_table):
    """get_shocks labour draw (AS:1245-1256) given the uniforms the global RNG would give:
    l' = searchsorted(cdf[l], u, 'right')."""
    out = np.empty(lab_prev.size, dtype=np.int64)
    for l in range(cdf_table.shape[0]):
        sel = lab_prev == l
        out[sel] = np.searchsorted(cdf_table[l], u[sel], side="right")
    return out


def sim_one_period(a_prev, lab_prev, emp, u, Rnow, Wnow, Mnow, Mrkv, LSStates, cdf_table,
                   m_tab, c_tab, Mgrid):
    """One [HARK] sim_one_period: get_shocks -> get_states -> get_controls -> get_poststates
    (AS:1217-1415).  Returns (a_now, lab_now, m_now, c_now)."""
    lab_now = draw_labor(lab_prev, u, cdf_table)
    IdioLS = LSStates[lab_now]
    EmpF = emp.astype(np.float64)
    mNow = Rnow * a_prev + Wnow * np.multiply(IdioLS, EmpF)                  # AS:1283
    cNow = np.zeros(a_prev.size)
    state = 4 * lab_now + 2 * int(Mrkv) + emp.astype(np.int64)               # AS:1326-1356
    with np.errstate(all="ignore"):
        for s in np.unique(state):
            sel = state == s
            cNow[sel] = eval_policy_2d(m_tab, c_tab, Mgrid, int(s), mNow[sel], Mnow)
    aNow = mNow - cNow                                                       # AS:1415
    return aNow, lab_now, mNow, cNow


def calc_R_and_W(aNow, EmpNow, MrkvNow, e):
    """AiyagariEconomy.calc_R_and_W (AS:1839-1894).  Returns (Mnow, Aprev, Mrkv, Rnow, Wnow, Urate)."""
    Aprev = np.mean(np.array(aNow))
    AggK = Aprev
    Urate = 1.0 - np.mean(np.array(EmpNow))
    if MrkvNow == 0:
        Prod = e["ProdB"]
        AggL = (1.0 - e["UrateB"]) * e["LbrInd"]
    else:
        Prod = e["ProdG"]
        AggL = (1.0 - e["UrateG"]) * e["LbrInd"]
    KtoLnow = AggK / AggL
    Rnow = 1.0 + Prod * (e["CapShare"] * KtoLnow ** (e["CapShare"] - 1.0)) - e["DeprFac"]
    Wnow = Prod * ((1.0 - e["CapShare"]) * KtoLnow ** (e["CapShare"]))
    Mnow = Rnow * AggK + Wnow * AggL
    return Mnow, Aprev, MrkvNow, Rnow, Wnow, Urate


def calc_AFunc(Mnow_hist, Aprev_hist, MrkvNow_hist, e, intercept_prev, slope_prev):
    """AiyagariEconomy.calc_AFunc (AS:1896-1964).  Mutates intercept_prev / slope_prev in place
    (quirk Q9) and returns (AggShocksDynamicRule, r^2 list)."""
    discard = e["T_discard"]
    w = 1.0 - e["DampingFac"]
    T = len(Mnow_hist)
    logA = np.log(np.asarray(Aprev_hist)[discard:T])
    logM = np.log(np.asarray(Mnow_hist)[discard - 1:T - 1])
    hist = np.asarray(MrkvNow_hist)[discard - 1:T - 1]
    AFunc_list, rsq = [], []
    for i in range(2):
        these = i == hist
        res = stats.linregress(logM[these], logA[these])
        intercept = w * res.intercept + (1.0 - w) * intercept_prev[i]
        slope = w * res.slope + (1.0 - w) * slope_prev[i]
        AFunc_list.append(AggregateSavingRule(intercept, slope))
        rsq.append(res.rvalue ** 2)
        intercept_prev[i] = intercept
        slope_prev[i] = slope
    return AggShocksDynamicRule(AFunc_list), rsq


# --------------------------------------------------------------------------------------
# The whole GE fixed point (rows C1-C6)
# --------------------------------------------------------------------------------------
class KSModel:
    """Reference driver restated (AH:191-258): AiyagariEconomy + one AiyagariType.

    ``u_source(ge_iter, t0, t1)`` returns the uniforms [t1 - t0, AgentCount] the global
    ``np.random`` would feed ``np.random.choice`` (AS:1254) in that window."""

    def __init__(self, econ_dict=None, agent_dict=None):
        e = deepcopy(INIT_ECONOMY)
        e.update(econ_dict or {})
        a = dict(INIT_AGENTS)
        a.update(agent_dict or {})
        self.e, self.a = e, a
        self.ss = steady_state(e)
        mk = make_MrkvArray(e)
        self.MrkvArray, self.MrkvIndArray = mk["MrkvArray"], mk["MrkvIndArray"]
        self.MrkvEmplArray = mk["MrkvEmplArray"]
        self.econ_tauchen = mk["TauchenAux"]
        self.agent_tauchen = tauchen_for(a["LaborStatesNo"], a["LaborAR"], a["LaborSD"])   # Q5
        self.LSStates = labor_levels(self.agent_tauchen[0])
        self.cdf_table = np.array([choice_cdf(r) for r in self.agent_tauchen[1]])
        self.aGrid = make_grid_exp_mult(a["aMin"], a["aMax"], a["aCount"], a["aNestFac"])
        self.Mgrid = self.ss["MSS"] * np.asarray(a["MgridBase"])
        self.intercept_prev = list(e["intercept_prev"])
        self.slope_prev = list(e["slope_prev"])
        self.AFunc = [AggregateSavingRule(self.intercept_prev[j], self.slope_prev[j]) for j in range(2)]
        self.Mrkv_hist = make_Mrkv_history(self.MrkvArray, e["act_T"], e["MrkvNow_init"], seed=0)
        self.agent_seed = 0

    def solve_agent(self, tol=AGENT_TOLERANCE):
        Rk, Wk, Mk = next_prices(self.AFunc, self.Mgrid, self.a["LaborStatesNo"], self.e)
        return egm_solve(self.a["DiscFac"], self.a["CRRA"], self.aGrid, self.Mgrid, Rk, Wk, Mk,
                         self.LSStates, self.MrkvIndArray, tol=tol)

    def make_history(self, m_tab, c_tab, u_source, ge_iter=0, act_T=None, record=False):
        e = self.e
        T = act_T or e["act_T"]
        N = self.a["AgentCount"]
        emp, lab, rng = sim_birth_labor(N, self.a["LaborStatesNo"], e["UrateB"], seed=self.agent_seed,
                                        Mrkv=e["MrkvNow_init"], UrateG=e["UrateG"], return_rng=True)
        ks = e["UrateB"] != 0.0 or e["UrateG"] != 0.0     # else everyone stays employed
        perms = make_emp_idx_arrays(N, e["UrateB"], e["UrateG"], self.MrkvEmplArray, self.MrkvArray) if ks else None
        a_prev = np.full(N, self.ss["KSS"])
        sow = dict(Mnow=self.ss["MSS"], Aprev=self.ss["KSS"], Mrkv=0, Rnow=self.ss["RSS"], Wnow=self.ss["WSS"])
        hist = dict(Mrkv=[], Aprev=[], Mnow=[], Urate=[])
        trace = []
        block = 1000
        for t0 in range(0, T, block):
            t1 = min(T, t0 + block)
            U = u_source(ge_iter, t0, t1)
            for t in range(t0, t1):
                if ks:
                    emp = employment_step(emp, sow["Mrkv"], e["UrateB"], perms, rng)
                a_prev, lab, m_now, c_now = sim_one_period(a_prev, lab, emp, U[t - t0], sow["Rnow"], sow["Wnow"],
                                                           sow["Mnow"], sow["Mrkv"], self.LSStates, self.cdf_table,
                                                           m_tab, c_tab, self.Mgrid)
                Mnow, Aprev, Mrkv, Rnow, Wnow, Urate = calc_R_and_W([a_prev], [emp.astype(np.float64)],
                                                                   self.Mrkv_hist[t], e)
                sow = dict(Mnow=Mnow, Aprev=Aprev, Mrkv=Mrkv, Rnow=Rnow, Wnow=Wnow)
                hist["Mrkv"].append(Mrkv)
                hist["Aprev"].append(Aprev)
                hist["Mnow"].append(Mnow)
                hist["Urate"].append(Urate)
                if record:
                    trace.append((a_prev.copy(), lab.copy(), emp.copy()))
        return dict(sow=sow, hist=hist, aNow=a_prev, lab=lab, emp=emp, trace=trace)

    def solve(self, u_source, max_loops=MAX_LOOPS, tol=MARKET_TOLERANCE, log=None):
        """[HARK 0.12] Market.solve (C5)."""
        old = None
        completed = 0
        go = True
        out = None
        while go:
            m, c, cycles, dist_agent = self.solve_agent()
            out = self.make_history(m, c, u_source, ge_iter=completed)
            new, rsq = calc_AFunc(out["hist"]["Mnow"], out["hist"]["Aprev"], self.Mrkv_hist, self.e,
                                  self.intercept_prev, self.slope_prev)
            self.AFunc = new.AFunc
            distance = distance_metric(new, old) if completed > 0 else 1000000.0
            if log is not None:
                log.append(dict(iter=completed, cycles=cycles, intercept=list(self.intercept_prev),
                                slope=list(self.slope_prev), distance=distance, Rnow=out["sow"]["Rnow"]))
            old = new
            completed += 1
            go = distance >= tol and completed < max_loops
        self.result = out
        self.solution_tables = (m, c)
        return out

    def results(self):
        """AH:257-258: r = Rnow_T - 1; saving rate = delta K_T / (M_T - (1 - delta) K_T)."""
        sow = self.result["sow"]
        K = np.mean(self.result["aNow"])
        d = self.e["DeprFac"]
        return dict(r=sow["Rnow"] - 1.0, saving_rate=d * K / (sow["Mnow"] - (1 - d) * K), K=K)


def numpy_global_u_source(seed, N):
    """The uniforms the reference's unseeded global RNG would feed np.random.choice (AS:1254)
    had it been seeded with ``np.random.seed(seed)`` before ``econ.solve()``: one continuing
    MT19937 stream, agent-major within a period, periods in order, GE iterations in order
    (``RandomState.choice`` draws exactly one ``random_sample()`` per call)."""
    rng = np.random.RandomState(seed)

    def src(ge_iter, t0, t1):
        return rng.random_sample((t1 - t0, N))

    return src
