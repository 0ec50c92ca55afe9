"""Krusell-Smith employment mode at the calibration the reference's
comments give (UrateB = 0.10, UrateG = 0.04, ProdB = 0.99, ProdG = 1.01,
Aiyagari_Support.py:1538-1547) against the oracle, with the reference's global-RNG
labour stream seeded identically and the agent RNG's exact-count employment
permutations (AS:1042-1156, 1222-1240):

  * the employment of every agent in every period and the recorded Urate history are
    identical (the employment is drawn on the host with the agent RNG, as the reference
    draws it);
  * labour states identical; assets and the aggregate history within 1e-12 where finite
    and NaN in the same places.

The reference's KS branch is internally inconsistent: its household solve pays the
unemployed sub-states their labour income (AS:990-1018, the "#! KS: this must be zero!"
lines), while the simulation pays them nothing (AS:1283).  Unemployed agents therefore
run their assets down to the borrowing node, m = R a falls below HARK LinearInterp's
first node (1e-7, AS:1503-1504) and c = NaN within a few periods; from there the
aggregate history is NaN.  The device reproduces that behaviour, NaN for NaN."""
import numpy as np
import pytest
import torch

from oracle import hark_ks as H

pytestmark = pytest.mark.gpu

KS = dict(UrateB=0.10, UrateG=0.04, ProdB=0.99, ProdG=1.01)


def _economy(gpu, act_T, agents, engine="auto", history_engine="fused"):
    from aiyagari_hark_amd import AiyagariEconomy, AiyagariType
    econ = AiyagariEconomy(act_T=act_T, T_discard=50, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0], **KS)
    econ.verbose = False
    econ.history_engine = history_engine
    agent = AiyagariType(device=gpu, shock_mode="numpy", AgentCount=agents, panel_engine=engine)
    agent.cycles = 0
    agent.get_economy_data(econ)
    econ.agents = [agent]
    econ.make_Mrkv_history()
    return econ, agent


def _close_or_both_nan(got, want, rtol=1e-12, atol=1e-13):
    got, want = np.asarray(got, dtype=np.float64), np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], rtol=rtol, atol=atol)


@pytest.mark.parametrize("engine,history", [("block", "fused"), ("grid", "fused"), ("auto", "hooks")])
def test_ks_history_matches_oracle(gpu, engine, history):
    T, N = 120, 700
    econ, agent = _economy(gpu, T, N, engine, history)
    agent.solve()
    np.random.seed(5)
    econ.make_history()
    ref = H.KSModel(dict(act_T=T, T_discard=50, **KS), dict(AgentCount=N))
    m, c, _, _ = ref.solve_agent()
    out = ref.make_history(m, c, H.numpy_global_u_source(5, N))
    np.testing.assert_array_equal(np.asarray(econ.history["Mrkv"]), np.asarray(out["hist"]["Mrkv"]))
    np.testing.assert_array_equal(np.asarray(econ.history["Urate"]), np.asarray(out["hist"]["Urate"]))
    assert set(np.round(np.asarray(out["hist"]["Urate"]) * N).astype(int)) == {28, 70}   # exact counts
    np.testing.assert_array_equal(np.asarray(econ.reap_state["EmpNow"][0]).astype(bool), out["emp"])
    lab = agent.state_now["LaborSupplyState"]
    lab = lab.cpu().numpy() if torch.is_tensor(lab) else np.asarray(lab)   # device-resident on the hooks path
    np.testing.assert_array_equal(lab.astype(np.int64), out["lab"])
    _close_or_both_nan(econ.history["Aprev"], out["hist"]["Aprev"])
    _close_or_both_nan(econ.history["Mnow"], out["hist"]["Mnow"])
    _close_or_both_nan(econ.reap_state["aNow"][0], out["aNow"])
    # the reference's KS branch goes NaN (module docstring): both do, at the same period
    first = int(np.argmax(~np.isfinite(np.asarray(out["hist"]["Aprev"], dtype=np.float64))))
    assert 0 < first < T


def test_ks_ge_loop_matches_oracle(gpu):
    """Market.solve in KS mode: the same number of GE iterations and the same (NaN)
    saving rules as the oracle's fixed-point loop (a NaN distance ends the loop,
    `distance >= tolerance` being False)."""
    T, N = 150, 700
    econ, agent = _economy(gpu, T, N)
    np.random.seed(9)
    econ.solve()
    ref = H.KSModel(dict(act_T=T, T_discard=50, **KS), dict(AgentCount=N))
    log = []
    ref.solve(H.numpy_global_u_source(9, N), log=log)
    assert len(econ.ge_log) == len(log)
    for g, o in zip(econ.ge_log, log):
        assert g["cycles"] == o["cycles"]
        np.testing.assert_allclose(g["intercept"], o["intercept"], rtol=1e-9, atol=1e-12)   # NaN == NaN
        np.testing.assert_allclose(g["slope"], o["slope"], rtol=1e-9, atol=1e-12)


def test_ks_tables_have_unemployed_cells(gpu):
    """aiy_panel_build with the unemployed sub-states: the unemployed cells' policy is the
    EGM's unemployed rows (c at m for s = 4 l + 2 g + 0), checked through a one-period
    panel of unemployed agents against the oracle's policy evaluation."""
    from aiyagari_hark_amd import _lib
    from aiyagari_hark_amd.panel import DevicePanel
    econ, agent = _economy(gpu, 20, 700)
    agent.solve()
    sol = agent.solution[0]
    N = 700
    p = DevicePanel(N, device=gpu, act_T=20, engine="grid")
    lvl = torch.as_tensor(agent.LSStates, dtype=torch.float64).to(gpu)
    cdf = torch.as_tensor(np.eye(7).cumsum(axis=1), dtype=torch.float64).to(gpu)   # labour state kept
    hist = torch.zeros(20, dtype=torch.int32, device=gpu)
    p.bind_model(sol.m_tab, sol.c_tab, sol.M_grid, lvl, cdf, hist, econ.market_constants(), unemployed=True)
    a0 = np.linspace(0.05, 30.0, N)
    lab0 = np.arange(N) % 7
    emp0 = (np.arange(N) % 3 != 0).astype(np.uint8)
    p.reset(a0, lab0, econ.MSS, econ.KSS, 0, econ.RSS, econ.WSS)
    p.run(0, 1, shock_mode="numpy", u_host_source=lambda n: np.full((n, N), 0.5), emp_source=lambda n: emp0[None])
    torch.cuda.synchronize()
    m = econ.RSS * a0 + econ.WSS * (agent.LSStates[lab0] * emp0)
    s = 4 * lab0 + 0 + emp0
    want = np.empty(N)
    mt, ct, Mg = sol.m_host(), sol.c_host(), sol.M_grid_host()
    for k in np.unique(s):
        sel = s == k
        want[sel] = m[sel] - H.eval_policy_2d(mt, ct, Mg, int(k), m[sel], float(econ.MSS))
    _close_or_both_nan(p.a.cpu().numpy(), want)
    with pytest.raises(ValueError):   # employment states need the unemployed tables
        q = DevicePanel(N, device=gpu, act_T=20, engine="grid")
        q.bind_model(sol.m_tab, sol.c_tab, sol.M_grid, lvl, cdf, hist, econ.market_constants())
        q.reset(a0, lab0, econ.MSS, econ.KSS, 0, econ.RSS, econ.WSS)
        q.run(0, 1, shock_mode="philox", emp_source=lambda n: emp0[None])
    h = _lib.handle(gpu.index)
    assert h.lib.aiy_panel_table_bytes(7, 15, 32, 1) > h.lib.aiy_panel_table_bytes(7, 15, 32, 0)
