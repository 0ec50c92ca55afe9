"""The reference's per-period simulation hooks (AiyagariType.get_shocks / get_states /
get_controls / get_poststates / sim_one_period / simulate / market_action and the Market's
sow / cultivate / reap / mill / store, AS:1161, 1217-1415, [HARK] Market.make_history)
driven one at a time through the C ABI (aiy_get_* / aiy_sum), checked against the fused
history kernel (aiy_sim_periods) on the same shocks: labour draws bit for bit, assets and
the aggregate history to 1e-12 relative (only the summation order of the per-period mean
differs)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _economy(gpu, shock_mode, agents=700, act_T=240):
    from aiyagari_hark_amd import AiyagariEconomy, AiyagariType
    econ = AiyagariEconomy(act_T=act_T, T_discard=60, intercept_prev=[0.0, 0.0], slope_prev=[1.0, 1.0])
    econ.verbose = False
    agent = AiyagariType(device=gpu, shock_mode=shock_mode, shock_seed=11, AgentCount=agents)
    agent.cycles = 0
    agent.get_economy_data(econ)
    econ.agents = [agent]
    econ.make_Mrkv_history()
    return econ, agent


def _history(econ, engine, seed=None):
    econ.history_engine = engine
    if seed is not None:
        np.random.seed(seed)
    econ.make_history()
    torch.cuda.synchronize()
    lab = econ.agents[0].state_now["LaborSupplyState"]
    lab = lab.cpu().numpy() if torch.is_tensor(lab) else np.asarray(lab)
    return dict(a=np.asarray(econ.reap_state["aNow"][0], dtype=np.float64), lab=lab.astype(np.int64),
                A=np.asarray(econ.history["Aprev"], dtype=np.float64), M=np.asarray(econ.history["Mnow"]),
                Mrkv=np.asarray(econ.history["Mrkv"]), R=econ.sow_state["Rnow"], W=econ.sow_state["Wnow"])


@pytest.mark.parametrize("shock_mode", ["philox", "numpy"])
def test_hooks_history_equals_fused(gpu, shock_mode):
    econ, agent = _economy(gpu, shock_mode)
    agent.solve()
    fused = _history(econ, "fused", seed=5)
    hooks = _history(econ, "hooks", seed=5)
    np.testing.assert_array_equal(hooks["lab"], fused["lab"])
    np.testing.assert_array_equal(hooks["Mrkv"], fused["Mrkv"])
    np.testing.assert_allclose(hooks["a"], fused["a"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(hooks["A"], fused["A"], rtol=1e-12)
    np.testing.assert_allclose(hooks["M"], fused["M"], rtol=1e-12)
    assert abs(hooks["R"] - fused["R"]) < 1e-13 and abs(hooks["W"] - fused["W"]) < 1e-12


def test_hooks_ge_loop_matches_fused(gpu):
    """Two KS fixed-point iterations with the period loop on the host give the fused
    path's saving rules."""
    rules = {}
    for engine in ("fused", "hooks"):
        econ, agent = _economy(gpu, "philox", agents=350, act_T=200)
        econ.history_engine = engine
        econ.max_loops = 2
        econ.solve()
        rules[engine] = (list(econ.intercept_prev), list(econ.slope_prev))
    np.testing.assert_allclose(rules["hooks"][0], rules["fused"][0], rtol=1e-10, atol=1e-12)
    np.testing.assert_allclose(rules["hooks"][1], rules["fused"][1], rtol=1e-10, atol=1e-12)


def test_simulate_and_market_action(gpu):
    """AgentType.simulate(n) == n market_action() calls == n sim_one_period() calls at
    fixed prices (the sown Rnow / Wnow / Mnow / Mrkv)."""
    out = []
    for how in ("simulate", "market_action", "sim_one_period"):
        econ, agent = _economy(gpu, "philox", agents=700)
        agent.solve()
        econ.reset()
        econ.sow()
        if how == "simulate":
            agent.simulate(5)
        else:
            for _ in range(5):
                getattr(agent, how)()
        torch.cuda.synchronize()
        assert agent.t_sim == 5
        out.append((agent.state_now["aNow"].cpu().numpy(), agent.state_now["LaborSupplyState"].cpu().numpy()))
    for a, lab in out[1:]:
        np.testing.assert_array_equal(a, out[0][0])
        np.testing.assert_array_equal(lab, out[0][1])
    # a = m - c with c = cFunc(m, Mnow) of the agent's labour state (HARK evaluation)
    agent_a = out[0][0]
    assert np.all(np.isfinite(agent_a)) and np.all(agent_a > 0)


def test_hook_entry_points_reject_bad_arguments(gpu):
    from aiyagari_hark_amd import _lib
    h = _lib.handle(gpu.index)
    lab = torch.zeros(8, dtype=torch.uint8, device=gpu)
    cdf = torch.ones(1, dtype=torch.float64, device=gpu)
    s = _lib.stream_ptr()
    assert h.lib.aiy_get_shocks(h.h, 0, _lib.ptr(cdf), 8, 0, _lib.ptr(lab), None, 0, 0, 0, s) == -1
    assert h.lib.aiy_get_shocks(h.h, 1, _lib.ptr(cdf), 8, 0, _lib.ptr(lab), None, 0, 1 << 12, 0, s) == -1
    assert h.lib.aiy_get_controls(h.h, 6, 1, 4, None, None, None, 0, 1.0, 8, None, None, None, None, s) == -1
    assert h.lib.aiy_get_controls(h.h, 8, 1, 4, None, None, None, 2, 1.0, 8, None, None, None, None, s) == -1
    assert h.lib.aiy_sum(h.h, None, 4, None, s) == -1
    out = torch.full((1,), 7.0, dtype=torch.float64, device=gpu)
    assert h.lib.aiy_sum(h.h, None, 0, _lib.ptr(out), s) == 0
    torch.cuda.synchronize()
    assert float(out.item()) == 0.0
