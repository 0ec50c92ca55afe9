"""GPU parity at the BENCHMARKED size of configs[1]: the
10 000-point asset grid (28 states x 15 M nodes) and the 1 000 006-agent panel, against
the CPU oracle on the same inputs.

* one EGM step at N_a = 10 000, bit-exact (CRRA = 1: the kernel follows NumPy's operation
  order, Aiyagari_Support.py:1478-1504);
* the converged 10 000-point solve ([HARK] solve_agent, tol 1e-6, cold start): the same
  cycle count and tables within 1e-8 relative (north_star);
* 20 periods of the 1 000 006-agent persistent panel with host uniforms against
  oracle.sim_one_period + calc_R_and_W (Aiyagari_Support.py:1217-1415, 1839-1894):
  labour states exact, assets and the K / M history to 1e-12;
* the streaming form of the persistent kernel (agents in HBM, the form panels above ~4M
  agents take: configs[3] shards) against the one-launch-per-period kernel.
"""
import numpy as np
import pytest
import torch

from oracle import hark_ks as H

pytestmark = pytest.mark.gpu
N_A = 10_000
N_AGENTS = 1_000_006


@pytest.fixture(scope="module")
def big():
    m = H.KSModel(dict(act_T=60), dict(aCount=N_A, AgentCount=N_AGENTS))
    Rk, Wk, Mk = H.next_prices(m.AFunc, m.Mgrid, 7, m.e)
    args = (0.96, 1.0, m.aGrid, m.Mgrid, Rk, Wk, Mk, m.LSStates, m.MrkvIndArray)
    return m, (Rk, Wk, Mk), args


@pytest.fixture(scope="module")
def solved(big, gpu):
    """Oracle and device converged 10k solutions (the oracle takes ~30 s on one core)."""
    from aiyagari_hark_amd.egm import EgmBatch, egm_solve
    m, (Rk, Wk, Mk), args = big
    mo, co, cyc_o, dist_o = H.egm_solve(*args)
    lab = np.array([m.LSStates[s // 4] for s in range(28)])
    b = EgmBatch.from_numpy(m.aGrid, m.Mgrid, m.MrkvIndArray, Rk, Wk, Mk, lab, 0.96, 1.0, device=gpu)
    md, cd, cyc_d, dist_d = egm_solve(b, tol=1e-6, max_cycles=5000)
    return dict(mo=mo, co=co, cyc_o=cyc_o, dist_o=dist_o, md=md[0], cd=cd[0], cyc_d=int(cyc_d[0]),
                dist_d=float(dist_d[0]), batch=b)


@pytest.mark.timeout(300)
def test_egm_step_10k_bit_exact(big, gpu):
    from aiyagari_hark_amd.egm import EgmBatch, egm_step
    m, (Rk, Wk, Mk), args = big
    m1, c1 = H.egm_step(None, None, *args)
    m2, c2 = H.egm_step(m1, c1, *args)
    m3, c3 = H.egm_step(m2, c2, *args)
    lab = np.array([m.LSStates[s // 4] for s in range(28)])
    b = EgmBatch.from_numpy(m.aGrid, m.Mgrid, m.MrkvIndArray, Rk, Wk, Mk, lab, 0.96, 1.0, device=gpu)
    dev = lambda x: torch.as_tensor(x[None]).to(gpu)
    # no row hints yet (global searches), then hints from the cycle before (as in a
    # solve), then hints from the same tables (the window path everywhere)
    for tables, (wm, wc) in (((m1, c1), (m2, c2)), ((m2, c2), (m3, c3)), ((m2, c2), (m3, c3))):
        om, oc = egm_step(b, dev(tables[0]), dev(tables[1]))
        assert np.array_equal(oc[0].cpu().numpy(), wc)
        assert np.array_equal(om[0].cpu().numpy(), wm)


@pytest.mark.timeout(600)
def test_egm_solve_10k_same_cycles(solved):
    s = solved
    assert s["cyc_d"] == s["cyc_o"]
    c = s["cd"].cpu().numpy()
    mm = s["md"].cpu().numpy()
    assert np.max(np.abs(c - s["co"]) / np.abs(s["co"])) <= 1e-8
    assert np.max(np.abs(mm - s["mo"]) / np.abs(s["mo"])) <= 1e-8
    assert s["dist_d"] == pytest.approx(s["dist_o"], rel=1e-6)


def _panel(gpu, m, md, cd, b, T):
    from aiyagari_hark_amd.panel import DevicePanel
    p = DevicePanel(N_AGENTS, device=gpu, act_T=T, engine="grid")
    p.bind_model(md, cd, b.M_grid[0], torch.as_tensor(m.LSStates).to(gpu), torch.as_tensor(m.cdf_table).to(gpu),
                 torch.as_tensor(m.Mrkv_hist[:T].astype(np.int32)).to(gpu),
                 dict(CapShare=0.36, DeprFac=0.08, prod=(1.0, 1.0), agg_L=(1.0, 1.0)))
    return p


@pytest.mark.timeout(600)
def test_resident_panel_1M_agents_host_uniforms(big, solved, gpu):
    m = big[0]
    T = 20
    md, cd = solved["md"], solved["cd"]
    emp, lab0 = H.sim_birth_labor(N_AGENTS, 7, 0.0, seed=0)
    U = np.random.RandomState(3).random_sample((T, N_AGENTS))
    p = _panel(gpu, m, md, cd, solved["batch"], T)
    p.reset(m.ss["KSS"], lab0, m.ss["MSS"], m.ss["KSS"], 0, m.ss["RSS"], m.ss["WSS"])
    pos = {"t": 0}

    def src(n):
        o = U[pos["t"]:pos["t"] + n]
        pos["t"] += n
        return o

    p.run(0, T, shock_mode="numpy", u_host_source=src, chunk=T)   # one persistent launch
    torch.cuda.synchronize()
    mt, ct = md.cpu().numpy(), cd.cpu().numpy()   # the oracle simulates the same policy
    a = np.full(N_AGENTS, m.ss["KSS"])
    lab = lab0.copy()
    sow = (m.ss["MSS"], 0, m.ss["RSS"], m.ss["WSS"])
    hA, hM = [], []
    for t in range(T):
        a, lab, _, _ = H.sim_one_period(a, lab, emp, U[t], sow[2], sow[3], sow[0], sow[1], m.LSStates, m.cdf_table,
                                        mt, ct, m.Mgrid)
        Mn, Ap, Mr, Rn, Wn, _ = H.calc_R_and_W([a], [np.ones(N_AGENTS)], m.Mrkv_hist[t], m.e)
        sow = (Mn, Mr, Rn, Wn)
        hA.append(Ap)
        hM.append(Mn)
    assert np.array_equal(p.lab.cpu().numpy(), lab)
    ad = p.a.cpu().numpy()
    assert np.max(np.abs(ad - a)) / np.max(np.abs(a)) < 1e-12
    assert np.max(np.abs(p.hist_A.cpu().numpy() - np.array(hA)) / np.array(hA)) < 1e-12
    assert np.max(np.abs(p.hist_M.cpu().numpy() - np.array(hM)) / np.array(hM)) < 1e-12
    assert float(p.sow[3]) == pytest.approx(sow[2], rel=1e-12)


def test_streaming_resident_kernel_1M_agents(big, solved, gpu):
    """AIY_OPT_RESIDENT_STREAM forces the persistent kernel's HBM-streaming form
    (sim_resident_kernel<1024, 4, IN_LDS = false>, agent pairs per lane, the configs[3]
    shape) at the configs[1] population; it must equal the one-launch-per-period kernel
    (labour exact, assets / history to 1e-12) and be reproducible run to run."""
    from aiyagari_hark_amd import _lib
    m = big[0]
    T, seed = 30, 17
    md, cd = solved["md"], solved["cd"]
    _, lab0 = H.sim_birth_labor(N_AGENTS, 7, 0.0, seed=0)
    h = _lib.handle(gpu.index)
    out = {}
    try:
        for name, resident, stream in (("stream", 1, 1), ("period", 0, 0), ("lds", 1, 0), ("stream2", 1, 1)):
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT, resident), "opt")
            h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT_STREAM, stream), "opt")
            p = _panel(gpu, m, md, cd, solved["batch"], T)
            p.reset(m.ss["KSS"], lab0, m.ss["MSS"], m.ss["KSS"], 0, m.ss["RSS"], m.ss["WSS"])
            p.run(0, T, shock_mode="philox", seed=seed, ge_iter=0)
            torch.cuda.synchronize()
            out[name] = (p.lab.cpu().numpy(), p.a.cpu().numpy(), p.hist_A.cpu().numpy(), p.hist_M.cpu().numpy())
    finally:
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT, 1), "opt")
        h.check(h.lib.aiy_set_option(h.h, _lib.AIY_OPT_RESIDENT_STREAM, 0), "opt")
    ref = out["period"]
    for name in ("stream", "lds"):
        lab, a, hA, hM = out[name]
        assert np.array_equal(lab, ref[0]), name
        assert np.max(np.abs(a - ref[1])) / np.max(np.abs(ref[1])) < 1e-12, name
        assert np.max(np.abs(hA - ref[2]) / ref[2]) < 1e-12, name
        assert np.max(np.abs(hM - ref[3]) / ref[3]) < 1e-12, name
    for k in range(4):
        assert np.array_equal(out["stream"][k], out["stream2"][k])
