"""Host-side setup numerics.

These run once per calibration or once per GE iteration on tiny arrays (at most
S x S or n_M x S), so they stay on the host in NumPy/SciPy, exactly as the reference
computes them; everything per grid point or per agent runs in libaiyagari.

Citations: AS = /root/reference/Aiyagari_Support.py, [HARK] = econ-ark 0.12.
"""
from __future__ import annotations

import numpy as np
from scipy import special

MGRID_BASE = np.array([0.1, 0.3, 0.6, 0.8, 0.9, 0.95, 0.98, 1.0, 1.02, 1.05, 1.1, 1.2, 1.6, 2.0, 3.0])


def make_grid_exp_mult(ming, maxg, ng, timestonest=20):
    """Multi-exponential grid ([HARK] utilities.make_grid_exp_mult; AS:880)."""
    if timestonest > 0:
        lo, hi = ming, maxg
        for _ in range(timestonest):
            lo = np.log(lo + 1)
            hi = np.log(hi + 1)
        g = np.linspace(lo, hi, ng)
        for _ in range(timestonest):
            g = np.exp(g) - 1
        return g
    lo, hi = np.log(ming), np.log(maxg)
    return np.exp(np.arange(lo, hi + 0.000001, (hi - lo) / (ng - 1)))


def tauchen(n, sigma, rho, bound=3.0):
    """[HARK] distribution.make_tauchen_ar1(n, sigma, rho, bound) (AS:887, AS:1696)."""
    top = bound * sigma / ((1 - rho ** 2) ** 0.5)
    y = np.linspace(-top, top, n)
    d = y[1] - y[0]
    cdf = special.ndtr   # = stats.norm.cdf (scipy's norm._cdf is ndtr), without the per-call overhead
    # every (j, k) at once, each element by the same operations in the same order as HARK's
    # double loop (the Table II sweep builds 24 of these per step: 1.4 ms as scalar loops)
    yj, yk = y[:, None], y[None, :]
    hi = cdf((yk + d / 2.0 - rho * yj) / sigma)
    lo = cdf((yk - d / 2.0 - rho * yj) / sigma)
    P = hi - lo
    P[:, 0] = hi[:, 0]
    P[:, n - 1] = 1.0 - lo[:, n - 1]
    return y, P


def labor_tauchen(n_lab, labor_ar, labor_sd):
    """AS:885-887: innovation s.d. = LaborSD * sqrt(1 - LaborAR^2), bound 3."""
    return tauchen(n_lab, labor_sd * (1 - labor_ar ** 2) ** 0.5, labor_ar, 3.0)


def rouwenhorst(n, rho, sigma_y):
    """Rouwenhorst discretisation with unconditional s.d. sigma_y (build-defined E3)."""
    if n == 1:
        return np.zeros(1), np.ones((1, 1))
    p = (1.0 + rho) / 2.0
    P = np.array([[p, 1.0 - p], [1.0 - p, p]])
    for m in range(3, n + 1):
        Z = np.zeros((m, m))
        Z[:-1, :-1] += p * P
        Z[:-1, 1:] += (1.0 - p) * P
        Z[1:, :-1] += (1.0 - p) * P
        Z[1:, 1:] += p * P
        Z[1:-1, :] /= 2.0
        P = Z
    psi = np.sqrt(n - 1) * sigma_y
    return np.linspace(-psi, psi, n), P


def labor_levels(y):
    """exp(y) / mean(exp(y)) -- simple mean, not the stationary mean (AS:985, quirk Q3)."""
    ey = np.exp(y)
    return ey / np.mean(ey)


def steady_state(CRRA, DiscFac, DeprFac, CapShare, LbrInd):
    """AiyagariEconomy.update closed forms (AS:1606-1615)."""
    KtoL = ((1.0 ** CRRA / DiscFac - (1.0 - DeprFac)) / CapShare) ** (1.0 / (CapShare - 1.0))
    K = KtoL * LbrInd
    W = (1.0 - CapShare) * KtoL ** CapShare
    R = 1.0 + CapShare * KtoL ** (CapShare - 1.0) - DeprFac
    return dict(KtoLSS=KtoL, KSS=K, WSS=W, RSS=R, MSS=K * R + W * LbrInd, KtoYSS=KtoL ** (1.0 - CapShare))


def employment_chain(DurMeanB, DurMeanG, SpellMeanB, SpellMeanG, UrateB, UrateG, RelProbBG, RelProbGB):
    """MrkvAggArray [2,2] and MrkvEmplArray [4,4] in order BU, BE, GU, GE (AS:1647-1683)."""
    pBG, pGB = 1.0 / DurMeanB, 1.0 / DurMeanG
    pBB, pGG = 1.0 - pBG, 1.0 - pGB
    agg = np.array([[pBB, pBG], [pGB, pGG]])
    E = np.zeros((4, 4))
    E[0, 1] = pBB * 1.0 / SpellMeanB
    E[0, 0] = pBB * (1 - 1.0 / SpellMeanB)
    E[1, 0] = UrateB / (1.0 - UrateB) * E[0, 1]
    E[1, 1] = pBB - E[1, 0]
    E[2, 3] = pGG * 1.0 / SpellMeanG
    E[2, 2] = pGG * (1 - 1.0 / SpellMeanG)
    E[3, 2] = UrateG / (1.0 - UrateG) * E[2, 3]
    E[3, 3] = pGG - E[3, 2]
    E[0, 2] = RelProbBG * E[2, 2] / pGG * pBG
    E[0, 3] = pBG - E[0, 2]
    E[1, 2] = (pBG * UrateG - UrateB * E[0, 2]) / (1.0 - UrateB)
    E[1, 3] = pBG - E[1, 2]
    E[2, 0] = RelProbGB * E[0, 0] / pBB * pGB
    E[2, 1] = pGB - E[2, 0]
    E[3, 0] = (pGB * UrateB - UrateG * E[2, 0]) / (1.0 - UrateG)
    E[3, 1] = pGB - E[3, 0]
    return agg, E


def kron_states(P_lab, E):
    """MrkvIndArray: block (i, j) = P_lab[i, j] * E (AS:1715-1780), state s = 4 i + e."""
    n = P_lab.shape[0]
    out = np.empty((4 * n, 4 * n))
    for i in range(n):
        for j in range(n):
            out[4 * i:4 * i + 4, 4 * j:4 * j + 4] = np.array([row * P_lab[i, j] for row in E])
    if not np.all(out >= 0.0):
        raise AssertionError("Invalid idiosyncratic transition probabilities!")  # AS:1783-1785
    return out


def markov_history(MrkvArray, act_T, init=0, seed=0):
    """make_Mrkv_history (AS:1793-1805): [HARK] MarkovProcess(seed=0).draw, i.e.
    RandomState(0).choice(n, p=row) per period."""
    rng = np.random.RandomState(seed)
    out = np.zeros(act_T, dtype=int)
    now = init
    for t in range(act_T):
        out[t] = now
        now = rng.choice(MrkvArray.shape[1], p=MrkvArray[now, :])
    return out


def agg_state(S):
    """g(s') = (s' mod 4) div 2: KnextB, KnextB, KnextG, KnextG per labour state (AS:927)."""
    return (np.arange(S) % 4) // 2


def next_prices(intercepts, slopes, Mgrid, S, UrateB, UrateG, LbrInd, ProdB, ProdG, CapShare, DeprFac):
    """precompute_arrays (AS:923-976) without the redundant a and s axes:
    R[k, s'], W[k, s'], M'[k, s'] for next-period aggregate state g(s')."""
    g = agg_state(S)
    A = [np.exp(intercepts[j] + slopes[j] * np.log(Mgrid)) for j in range(2)]   # AFunc (AS:2004)
    K = np.where(g[None, :] == 0, A[0][:, None], A[1][:, None])
    L = np.where(g == 0, (1.0 - UrateB) * LbrInd, (1.0 - UrateG) * LbrInd)[None, :] * np.ones_like(K)
    Z = np.where(g == 0, ProdB, ProdG)[None, :] * np.ones_like(K)
    KtoL = K / L
    R = 1.0 + Z * CapShare * KtoL ** (CapShare - 1.0) - DeprFac
    W = Z * (1.0 - CapShare) * KtoL ** CapShare
    Y = Z * K ** CapShare * L ** (1.0 - CapShare)
    M = (1.0 - DeprFac) * K + Y
    return R, W, M


def choice_cdf_table(P):
    """Rows of cumsum(p) / cumsum(p)[-1] -- what np.random.choice(n, p=row) inverts."""
    out = np.empty_like(P, dtype=np.float64)
    for i in range(P.shape[0]):
        c = np.asarray(P[i], dtype=np.float64).cumsum()
        c /= c[-1]
        out[i] = c
    return out


def birth_states(AgentCount, n_lab, UrateB, seed=0, Mrkv=0, UrateG=None, with_rng=False):
    """sim_birth (AS:1173-1214) after [HARK] reset_rng: RandomState(seed); employment
    permutation (unemployment count of the birth period's macro state), then the even
    labour split permuted (two RNG.permutation calls).  with_rng: also return the agent
    RNG, which the per-period employment permutations continue (AS:1239-1240)."""
    if AgentCount % n_lab != 0:
        raise ValueError("AgentCount must be a multiple of LaborStatesNo (AS:757, AS:1203)")
    if Mrkv not in (0, 1):
        raise ValueError("Illegal macroeconomic state: MrkvNow must be 0 or 1")   # AS:1191-1192
    rate = UrateB if Mrkv == 0 or UrateG is None else UrateG
    rng = np.random.RandomState(seed)
    unemp = int(np.round(rate * AgentCount))
    emp = np.concatenate([np.zeros(unemp, dtype=bool), np.ones(AgentCount - unemp, dtype=bool)])
    lab = np.repeat(np.arange(n_lab), AgentCount // n_lab)
    emp = rng.permutation(emp)
    lab = rng.permutation(lab)
    return (emp, lab, rng) if with_rng else (emp, lab)


def employment_transitions(AgentCount, UrateB, UrateG, MrkvEmplArray, MrkvAggArray):
    """make_emp_idx_arrays (AS:1042-1156): for each macro transition j -> k the 0/1 arrays
    whose permutations assign this period's employment to last period's employed
    ("emp") and unemployed ("unemp") agents, so each state's unemployment count is exact.
    stay counts = round(previous count x P(stay | j -> k)) with the reference's operand
    order; the movers make up the new state's count."""
    unemp = [int(np.round(UrateB * AgentCount)), int(np.round(UrateG * AgentCount))]
    emp = [AgentCount - unemp[0], AgentCount - unemp[1]]
    out = {"emp": [[None, None], [None, None]], "unemp": [[None, None], [None, None]]}
    for j in (0, 1):
        for k in (0, 1):
            stay_u = int(np.round(unemp[j] * MrkvEmplArray[2 * j, 2 * k] / MrkvAggArray[j, k]))
            stay_e = int(np.round(emp[j] * (MrkvEmplArray[2 * j + 1, 2 * k + 1]) / MrkvAggArray[j, k]))
            to_u, to_e = unemp[k] - stay_u, emp[k] - stay_e
            out["emp"][j][k] = np.r_[np.ones(stay_e, dtype=bool), np.zeros(to_u, dtype=bool)]
            out["unemp"][j][k] = np.r_[np.ones(to_e, dtype=bool), np.zeros(stay_u, dtype=bool)]
    return out


def employment_step(emp_prev, mrkv_now, UrateB, trans, rng):
    """get_shocks' employment update (AS:1222-1240): previous macro state from last
    period's unemployment rate (compared with UrateB as a float, AS:1227), then one
    permutation for the employed and one for the unemployed (agent RNG, in that order).
    A transition array whose length differs from its group raises, as the reference's
    boolean assignment does."""
    was = np.asarray(emp_prev, dtype=bool)
    mrkv_prev = int(((~was).sum() / float(was.size)) != UrateB)
    e_arr, u_arr = trans["emp"][mrkv_prev][int(mrkv_now)], trans["unemp"][mrkv_prev][int(mrkv_now)]
    n_e = int(was.sum())
    if e_arr.size != n_e or u_arr.size != was.size - n_e:
        raise ValueError(f"employment transition {mrkv_prev}->{int(mrkv_now)}: arrays of {e_arr.size}/{u_arr.size} "
                         f"for {n_e} employed / {was.size - n_e} unemployed agents (AgentCount does not give exact "
                         "counts for these unemployment rates)")
    now = np.empty(was.size, dtype=bool)
    now[was] = rng.permutation(e_arr)
    now[~was] = rng.permutation(u_arr)
    return now
