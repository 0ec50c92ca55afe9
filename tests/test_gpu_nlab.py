"""Generalised discretisation on the Krusell-Smith path (VERDICT r2
item 9): the reference hard-codes 7 Tauchen states (Aiyagari_Support.py:927, 935-967,
990-1018, 1295-1408, 1715-1780); the build takes any LaborStatesNo (S = 4 N_l household
states).  At N_l = 5 and 9 the device path is held to the oracle (oracle/hark_ks.py, whose
make_MrkvArray forms the N_l x N_l blocks of kron(P_tauchen, MrkvEmplArray) in the
reference's order):

* the converged household tables (28 -> 20 / 36 states x 15 M nodes x 33 nodes) within 1e-8
  relative with the same cycle count;
* the panel over 40 periods with the same host uniforms: labour states exact, assets and
  the K / M history to 1e-12;
* the Krusell-Smith GE loop with the same global-RNG shock stream: every GE iteration's
  saving-rule coefficients within 1e-9, r and K/Y within 1e-5.
"""
import numpy as np
import pytest
import torch

from oracle import hark_ks as H

pytestmark = pytest.mark.gpu
CASES = [(5, 350), (9, 351)]   # (LaborStatesNo, AgentCount: a multiple of it, AS:757)


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    ok = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), ok)
    return float(np.max(np.abs(a[ok] - b[ok]) / np.maximum(np.abs(b[ok]), 1e-300)))


def _cal(n_lab):
    return dict(LaborStatesNo=n_lab, LaborAR=0.6, LaborSD=0.2, CRRA=1.0)


@pytest.mark.parametrize("n_lab,agents", CASES)
def test_ks_egm_tables_general_nlab(gpu, n_lab, agents):
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    m = H.KSModel(_cal(n_lab), dict(_cal(n_lab), AgentCount=agents))
    S = 4 * n_lab
    assert m.MrkvIndArray.shape == (S, S)
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, n_lab, m.e)
    mo, co, cyc_o, _ = H.egm_solve(0.96, 1.0, m.aGrid, m.Mgrid, Rk, Wk, Mk, m.LSStates, m.MrkvIndArray)
    lab = np.array([m.LSStates[s // 4] for s in range(S)])
    b = EgmBatch.from_numpy(m.aGrid, m.Mgrid, m.MrkvIndArray, Rk, Wk, Mk, lab, 0.96, 1.0, device=gpu)
    md, cd, cyc_d, _ = egm_solve(b, tol=1e-6, max_cycles=5000)
    assert int(cyc_d[0]) == cyc_o
    assert rel(cd[0].cpu().numpy(), co) <= 1e-8
    assert rel(md[0].cpu().numpy(), mo) <= 1e-8


@pytest.mark.parametrize("n_lab,agents", CASES)
def test_ks_panel_general_nlab(gpu, n_lab, agents):
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    from aiyagari_hark_amd.panel import DevicePanel
    m = H.KSModel(_cal(n_lab), dict(_cal(n_lab), AgentCount=agents))
    S, T = 4 * n_lab, 40
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, n_lab, m.e)
    lab = np.array([m.LSStates[s // 4] for s in range(S)])
    b = EgmBatch.from_numpy(m.aGrid, m.Mgrid, m.MrkvIndArray, Rk, Wk, Mk, lab, 0.96, 1.0, device=gpu)
    md, cd, _, _ = egm_solve(b, tol=1e-6, max_cycles=5000)
    emp, lab0 = H.sim_birth_labor(agents, n_lab, 0.0, seed=0)
    U = np.random.RandomState(2).random_sample((T, agents))
    p = DevicePanel(agents, device=gpu, act_T=T)
    p.bind_model(md[0], cd[0], b.M_grid[0], torch.as_tensor(m.LSStates).to(gpu), torch.as_tensor(m.cdf_table).to(gpu),
                 torch.as_tensor(m.Mrkv_hist[:T].astype(np.int32)).to(gpu),
                 dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0)))
    p.reset(m.ss["KSS"], lab0, m.ss["MSS"], m.ss["KSS"], 0, m.ss["RSS"], m.ss["WSS"])
    pos = {"t": 0}

    def src(n):
        o = U[pos["t"]:pos["t"] + n]
        pos["t"] += n
        return o

    p.run(0, T, shock_mode="numpy", u_host_source=src, chunk=T)
    torch.cuda.synchronize()
    mt, ct = md[0].cpu().numpy(), cd[0].cpu().numpy()
    a = np.full(agents, m.ss["KSS"])
    lb = lab0.copy()
    sow = (m.ss["MSS"], 0, m.ss["RSS"], m.ss["WSS"])
    hA, hM = [], []
    for t in range(T):
        a, lb, _, _ = H.sim_one_period(a, lb, emp, U[t], sow[2], sow[3], sow[0], sow[1], m.LSStates, m.cdf_table, mt, ct,
                                       m.Mgrid)
        Mn, Ap, Mr, Rn, Wn, _ = H.calc_R_and_W([a], [np.ones(agents)], m.Mrkv_hist[t], m.e)
        sow = (Mn, Mr, Rn, Wn)
        hA.append(Ap)
        hM.append(Mn)
    assert np.array_equal(p.lab.cpu().numpy(), lb)
    assert rel(p.a.cpu().numpy(), a) < 1e-12
    assert rel(p.hist_A.cpu().numpy(), hA) < 1e-12
    assert rel(p.hist_M.cpu().numpy(), hM) < 1e-12


@pytest.mark.parametrize("n_lab,agents", CASES)
def test_ks_ge_loop_general_nlab(gpu, n_lab, agents):
    from aiyagari_hark_amd.model import AiyagariEconomy, AiyagariType
    econ_d = dict(_cal(n_lab), act_T=1200, T_discard=400, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0])
    agent_d = dict(_cal(n_lab), AgentCount=agents)
    ref = H.KSModel(dict(econ_d), dict(agent_d))
    log = []
    ref.solve(H.numpy_global_u_source(5, agents), log=log)
    want = ref.results()
    econ = AiyagariEconomy(**dict(econ_d, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0]))
    econ.verbose = False
    agent = AiyagariType(**agent_d)
    agent.cycles = 0
    agent.get_economy_data(econ)
    econ.agents = [agent]
    econ.make_Mrkv_history()
    np.random.seed(5)
    econ.solve()
    assert agent.solution[0].m_tab.shape[0] == 4 * n_lab
    assert len(econ.ge_log) == len(log)
    for g, o in zip(econ.ge_log, log):
        assert g["cycles"] == o["cycles"]
        assert np.allclose(g["intercept"], o["intercept"], rtol=1e-9, atol=1e-12)
        assert np.allclose(g["slope"], o["slope"], rtol=1e-9, atol=1e-12)
    r = econ.sow_state["Rnow"] - 1
    K = np.mean(econ.reap_state["aNow"][0])
    KtoY = K / (econ.sow_state["Mnow"] - (1 - 0.08) * K)
    assert abs(r - want["r"]) < 1e-5
    assert abs(KtoY - want["saving_rate"] / 0.08) < 1e-5
