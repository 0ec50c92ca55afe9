"""CPU tests of the oracle (oracle/): pinned to the reference's closed forms, NumPy's own
RNG semantics, published KAT vectors, and the committed golden fixtures."""
import os

import numpy as np
import pytest
from scipy import stats

from oracle import hark_ks as H
from oracle import philox as PX
from oracle import stationary as ST

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_steady_state_closed_forms():
    # KSS, MSS for config 1; RSS = 1 / beta
    ss = H.steady_state(H.INIT_ECONOMY)
    assert ss["KSS"] == pytest.approx(5.446807380113233, rel=1e-15)
    assert ss["MSS"] == pytest.approx(6.851881950575776, rel=1e-15)
    assert ss["RSS"] == pytest.approx(1 / 0.96, rel=1e-14)


def test_table2_identity():
    # s = delta K/Y = delta alpha / (r + delta); r = 4.1666 % -> 23.67 %
    r, a, d = 0.041666, 0.36, 0.08
    assert d * a / (r + d) == pytest.approx(0.2367, abs=5e-5)


def test_grid_and_tauchen():
    g = H.make_grid_exp_mult(0.001, 50.0, 32, 2)
    assert g[0] == pytest.approx(0.001, rel=1e-12) and g[-1] == pytest.approx(50.0, rel=1e-12)
    assert np.all(np.diff(g) > 0)
    y, P = H.tauchen_for(7, 0.6, 0.2)
    assert np.allclose(P.sum(1), 1.0, atol=1e-15)
    assert y[-1] == pytest.approx(3 * 0.2, rel=1e-12)     # yN = 3 sigma_y
    assert np.allclose(y, -y[::-1])


def test_markov_kron():
    mk = H.make_MrkvArray(H.INIT_ECONOMY)
    P7 = mk["TauchenAux"][1]
    E4 = mk["MrkvEmplArray"]
    assert np.array_equal(mk["MrkvIndArray"], np.kron(P7, E4))
    assert np.allclose(mk["MrkvIndArray"].sum(1), 1.0, atol=1e-14)
    assert np.allclose(mk["MrkvArray"], [[7 / 8, 1 / 8], [1 / 8, 7 / 8]])
    # Urate = 0: employed rows of each aggregate block carry the whole block probability
    assert E4[1, 0] == 0.0 and E4[3, 2] == 0.0


def test_linear_interp_semantics():
    f = H.LinearInterp([1.0, 2.0, 4.0], [10.0, 20.0, 30.0])
    out = f(np.array([0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0]))
    assert np.isnan(out[0])                          # below the grid: NaN (lower_extrap=False)
    assert np.allclose(out[1:], [10, 15, 20, 25, 30, 40])   # linear extrapolation above
    g = H.LinearInterpOnInterp1D([H.LinearInterp([0, 1], [0, 1]), H.LinearInterp([0, 1], [0, 2])], [1.0, 2.0])
    assert g(np.array([0.5, 0.5, 0.5]), np.array([1.0, 1.5, 3.0])).tolist() == [0.5, 0.75, 1.5]


def test_egm_literal_vs_vectorised_bit_identical():
    for crra in (1.0, 5.0):
        m = H.KSModel(dict(CRRA=crra, LaborAR=0.9, LaborSD=0.4), dict(CRRA=crra, LaborAR=0.9, LaborSD=0.4))
        m.AFunc = [H.AggregateSavingRule(0.3, 0.85), H.AggregateSavingRule(0.32, 0.84)]
        arr = H.precompute_arrays_ref(m.aGrid, m.Mgrid, m.AFunc, m.LSStates, m.MrkvIndArray, m.e)
        sol = H.terminal_solution(28, crra)
        Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, 7, m.e)
        mt = ct = None
        for _ in range(3):
            sol = H.solve_Aiyagari_ref(sol, 0.96, crra, m.aGrid, m.Mgrid, arr["mNextArray"], arr["MnextArray"],
                                       arr["ProbArray"], arr["RnextArray"], 7)
            mt, ct = H.egm_step(mt, ct, 0.96, crra, m.aGrid, m.Mgrid, Rk, Wk, Mk, m.LSStates, m.MrkvIndArray)
            mr, cr = H.solution_to_tables(sol)
            assert np.array_equal(mr, mt) and np.array_equal(cr, ct)


def test_solve_agent_literal_vs_vectorised():
    m = H.KSModel()
    arr = H.precompute_arrays_ref(m.aGrid, m.Mgrid, m.AFunc, m.LSStates, m.MrkvIndArray, m.e)
    sol, cyc, d = H.solve_agent_ref(0.96, 1.0, m.aGrid, m.Mgrid, arr, 7)
    mt, ct, cyc2, d2 = m.solve_agent()
    mr, cr = H.solution_to_tables(sol)
    assert cyc == cyc2 and d == d2
    assert np.array_equal(mr, mt) and np.array_equal(cr, ct)


def test_choice_restatement_matches_numpy_choice():
    # get_shocks (AS:1253-1254) uses np.random.choice(7, p=P[l]); the oracle replays it from
    # the same uniforms: compare against NumPy's own choice on identical RandomStates.
    y, P = H.tauchen_for(7, 0.9, 0.4)
    cdf = np.array([H.choice_cdf(r) for r in P])
    lab = np.random.RandomState(3).randint(0, 7, size=2000)
    r1, r2 = np.random.RandomState(99), np.random.RandomState(99)
    ref = np.array([r1.choice(range(7), size=None, replace=True, p=P[l]) for l in lab])
    u = r2.random_sample(lab.size)
    assert np.array_equal(H.draw_labor(lab, u, cdf), ref)


def test_mrkv_history_matches_markov_process_choice():
    agg = np.array([[7 / 8, 1 / 8], [1 / 8, 7 / 8]])
    h = H.make_Mrkv_history(agg, 3000, 0, seed=0)
    rng = np.random.RandomState(0)
    cdf = np.cumsum(agg, axis=1)
    now, ref = 0, []
    for _ in range(3000):
        ref.append(now)
        now = int(np.searchsorted(cdf[now] / cdf[now][-1], rng.random_sample(), side="right"))
    assert h.tolist() == ref
    assert 0.3 < h.mean() < 0.7


def test_birth_permutations():
    emp, lab = H.sim_birth_labor(700, 7, 0.0, seed=0)
    assert emp.all() and np.bincount(lab).tolist() == [100] * 7
    rng = np.random.RandomState(0)
    rng.permutation(np.ones(700, dtype=bool))
    assert np.array_equal(lab, rng.permutation(np.repeat(np.arange(7), 100)))


def test_philox_kat():
    # Random123 kat_vectors for philox4x32_10
    cases = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
             ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
             ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
              (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for c, k, want in cases:
        got = PX.philox4x32_10(*[np.array([v], dtype=np.uint32) for v in c], *k)
        assert [int(g[0]) for g in got] == list(want)
    u = PX.uniform(5, np.arange(100000), 42)
    assert 0 <= u.min() and u.max() < 1 and abs(u.mean() - 0.5) < 0.005


def test_linregress_is_scipy():
    x = np.log(np.linspace(5, 8, 100))
    y = 0.1 + 0.95 * x
    r = stats.linregress(x, y)
    assert r.slope == pytest.approx(0.95) and r.intercept == pytest.approx(0.1)


def test_golden_fixtures_reproduce():
    from tests.golden import make_golden as G
    fx = np.load(os.path.join(GOLD, "egm_cfg1.npz"))
    now = G.egm_fixture("cfg1")
    for k in ("m", "c", "P", "aGrid", "Mgrid", "Rk", "Wk", "Mk"):
        assert np.array_equal(fx[k], now[k]), k
    assert int(fx["cycles"]) == now["cycles"]
    p = np.load(os.path.join(GOLD, "panel_cfg1.npz"))
    pn = G.panel_fixture("cfg1")
    assert np.array_equal(p["hist_A"], pn["hist_A"]) and np.array_equal(p["lab_final"], pn["lab_final"])


def test_rouwenhorst_moments():
    y, P = ST.rouwenhorst(25, 0.9, 0.4)
    assert np.allclose(P.sum(1), 1.0, atol=1e-14)
    w, v = np.linalg.eig(P.T)
    pi = np.real(v[:, np.argmin(abs(w - 1))])
    pi /= pi.sum()
    mean = pi @ y
    var = pi @ (y - mean) ** 2
    assert var == pytest.approx(0.16, rel=1e-10)
    ac = (pi * (y - mean)) @ (P @ (y - mean)) / var
    assert ac == pytest.approx(0.9, rel=1e-10)


def test_stationary_lottery_conserves_mass():
    fx = np.load(os.path.join(GOLD, "stationary.npz"))
    assert fx["mass"].sum() == pytest.approx(1.0, abs=1e-12)
    assert fx["mass"].min() >= 0
    r = float(fx["r"])
    w, Kd = ST.prices(r, 0.36, 0.08)
    assert 0 < float(fx["K"]) < 50


def test_ge_short_run_oracle_anchor():
    """Reduced KS fixed point (act_T = 1500) runs, converges and stays near RSS."""
    m = H.KSModel(dict(act_T=1500, T_discard=500), dict(AgentCount=350))
    src = H.numpy_global_u_source(7, 350)
    log = []
    m.solve(src, log=log)
    res = m.results()
    assert len(log) >= 2
    assert 0.02 < res["r"] < 0.05
    assert res["saving_rate"] == pytest.approx(0.08 * 0.36 / (res["r"] + 0.08), rel=0.05)


def test_hark_utils_closed_form():
    """oracle/hark_utils.py on data 1..N: cum_data[k] = (k+1)(k+2) / (N (N+1))."""
    from oracle import hark_utils as HU
    x = np.arange(1.0, 11.0)
    rng = np.random.RandomState(0)
    shuffled = rng.permutation(x)
    assert abs(HU.get_lorenz_shares(shuffled, percentiles=[0.5])[0] - 30.0 / 110.0) < 1e-15
    assert abs(HU.get_lorenz_shares(shuffled, percentiles=[0.25])[0] - (6 + 0.5 * 6) / 110.0) < 1e-15
    assert abs(HU.get_percentiles(shuffled, percentiles=[0.5])[0] - 5.0) < 1e-12
    assert np.isnan(HU.get_percentiles(shuffled, percentiles=[0.05])[0])      # below cum_dist[0] = 0.1
    w = np.full(10, 2.0)
    assert abs(HU.get_lorenz_shares(shuffled, weights=w, percentiles=[0.5])[0] - 30.0 / 110.0) < 1e-15


@pytest.mark.parametrize("bad", [[0.0, 0.5], [0.5, 1.0], (0.2, 0.5)])
def test_wealth_stats_argument_checks(bad):
    """The device mirror rejects what HARK rejects, before touching the GPU."""
    from aiyagari_hark_amd import stats
    from oracle import hark_utils as HU
    for f in (stats.get_lorenz_shares, stats.get_percentiles, HU.get_lorenz_shares, HU.get_percentiles):
        with pytest.raises(ValueError):
            f(np.ones(5), percentiles=bad)


def test_brent_search_matches_scipy_brentq():
    """Host logic of the E1 root search (aiyagari_hark_amd.stationary._Brent): bisection
    until both signs are evaluated, then Brent's method -- the root scipy.optimize.brentq
    finds, to xtol, on monotone excess-demand-like functions."""
    from scipy.optimize import brentq
    from aiyagari_hark_amd.stationary import _Brent
    funcs = [lambda x: np.exp(40 * (x - 0.035)) - 1.0 - 3.0 * (0.03 - x),
             lambda x: (x - 0.0123) * (1.0 + 50 * x * x),
             lambda x: np.tanh(200 * (x + 0.01)) + 0.1 * x]
    for f in funcs:
        s = _Brent(-0.04, 0.0416, 1e-10)
        n = 0
        while not s.done and n < 100:
            s.update(f(s.propose()))
            n += 1
        want = brentq(f, -0.04, 0.0416, xtol=1e-12)
        assert abs(s.propose() - want) < 1e-9
        assert n < 40


def test_fast_hist_step_equals_reference_step():
    """The vectorised CPU bound (np.bincount) equals the np.add.at restatement."""
    from oracle import stationary as ST
    rng = np.random.default_rng(1)
    S, nA = 5, 300
    lo = np.sort(rng.integers(0, nA - 1, (S, nA)), axis=1)
    wlo = rng.random((S, nA))
    mass = rng.random((S, nA))
    mass /= mass.sum()
    P = rng.random((S, S))
    P /= P.sum(axis=1, keepdims=True)
    a = ST.hist_step(mass, lo, wlo, P)
    b = ST.hist_step_fast(mass, lo, wlo, P)
    assert np.max(np.abs(a - b)) < 1e-16


def test_employment_restatements_agree():
    """Krusell-Smith employment (AS:1042-1156, 1173-1214, 1222-1240): the product's host
    restatement (setup_math, drives the device panel) and the oracle's draw the same
    employment, period by period, from the same agent RNG; counts are exact per macro
    state; an AgentCount whose rounding breaks the counts raises."""
    from aiyagari_hark_amd import setup_math as sm
    p = dict(H.INIT_ECONOMY, UrateB=0.10, UrateG=0.04)
    mk = H.make_MrkvArray(p)
    E, A = mk["MrkvEmplArray"], mk["MrkvArray"]
    N = 700
    e1, l1, r1 = H.sim_birth_labor(N, 7, 0.10, seed=0, UrateG=0.04, return_rng=True)
    e2, l2, r2 = sm.birth_states(N, 7, 0.10, seed=0, UrateG=0.04, with_rng=True)
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_array_equal(l1, l2)
    perms = H.make_emp_idx_arrays(N, 0.10, 0.04, E, A)
    trans = sm.employment_transitions(N, 0.10, 0.04, E, A)
    hist = H.make_Mrkv_history(A, 300)
    for t in range(300):
        now = 0 if t == 0 else hist[t - 1]
        e1 = H.employment_step(e1, now, 0.10, perms, r1)
        e2 = sm.employment_step(e2, now, 0.10, trans, r2)
        np.testing.assert_array_equal(e1, e2)
        assert int((~e1).sum()) == (70 if now == 0 else 28)
    bad = 707   # round(0.04 * 707) etc. do not balance the flows
    tb = sm.employment_transitions(bad, 0.10, 0.04, E, A)
    eb, _, rb = sm.birth_states(bad, 7, 0.10, with_rng=True, UrateG=0.04)
    with pytest.raises(ValueError):
        for t in range(50):
            eb = sm.employment_step(eb, t % 2, 0.10, tb, rb)
