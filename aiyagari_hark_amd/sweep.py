"""Table II sweep in the reference's own algorithm (SURVEY.md §8 configs[2], rows A/B/C):
many (AiyagariEconomy, AiyagariType) pairs solved to their Krusell-Smith fixed point
together on one GPU.

The reference solves one calibration per notebook run (AH:191-258): set LaborAR,
LaborSD and CRRA in both dicts, ``econ.solve()``.  ``EconomyBatch.solve`` runs
[HARK] Market.solve for every economy of the batch in lock step:

    while any economy is active:
        solve_agents  -> ONE batched aiy_egm_solve over the active calibrations
                         (each stops on its own cycle, AS:1423 / [HARK] solve_agent)
        make_history  -> ONE aiy_sim_block_periods launch for all active panels
                         (a workgroup per calibration, agents in LDS, act_T periods)
        update_dynamics -> calc_AFunc per economy on the host (AS:1896-1964)
        an economy whose AFunc distance < tolerance leaves the batch

so each economy ends in exactly the state its own ``econ.solve()`` would leave
(sow_state, reap_state, history, dynamics, ge_log, agent.solution).  Shocks:
``"philox"`` keys each economy by its agent's ``shock_seed``; ``"numpy"`` gives each
economy its own ``RandomState(shock_seed)`` stream, equal to seeding the global RNG
with that seed before a single-economy solve (oracle.hark_ks.numpy_global_u_source).
"""
from __future__ import annotations

import numpy as np
import torch

from . import setup_math as sm
from .egm import EgmBatch, egm_solve
from .interp import DeviceSolution
from .panel import BatchedPanel


def table2_grid():
    """The 24 Table II cells (Aiyagari 1994): rho x sigma x CRRA."""
    return [dict(LaborAR=rho, LaborSD=sig, CRRA=mu) for rho in (0.0, 0.3, 0.6, 0.9) for sig in (0.2, 0.4)
            for mu in (1.0, 3.0, 5.0)]


def build_economies(cells, econ_dict=None, agent_dict=None, device=None, shock_mode="philox", seed0=0):
    """One (economy, agent) pair per cell, wired the way AH:225-241 wires them; the cell's
    LaborAR/LaborSD/CRRA go into both dicts (the notebook sets both from one variable)."""
    from .model import AiyagariEconomy, AiyagariType
    pairs = []
    for k, cell in enumerate(cells):
        e = dict(econ_dict or {})
        e.update(cell)
        e.setdefault("intercept_prev", [0.0, 0.0])
        e.setdefault("slope_prev", [1.0, 1.0])
        e["intercept_prev"] = list(e["intercept_prev"])
        e["slope_prev"] = list(e["slope_prev"])
        a = dict(agent_dict or {})
        a.update(cell)
        econ = AiyagariEconomy(**e)
        econ.verbose = False
        agent = AiyagariType(device=device, shock_mode=shock_mode, shock_seed=seed0 + k, **a)
        agent.cycles = 0
        agent.get_economy_data(econ)
        econ.agents = [agent]
        econ.make_Mrkv_history()
        pairs.append(econ)
    return pairs


class EconomyBatch:
    def __init__(self, economies, device=None):
        if not economies:
            raise ValueError("empty batch")
        self.econs = list(economies)
        self.agents = [e.agents[0] for e in self.econs]
        self.device = torch.device(device) if device is not None else self.agents[0].device
        a0 = self.agents[0]
        for e, a in zip(self.econs, self.agents):
            if len(e.agents) != 1:
                raise NotImplementedError("each economy has exactly one AgentType (AH:240)")
            same = (a.LaborStatesNo, a.aCount, len(a.MgridBase), a.AgentCount, e.act_T, a.shock_mode) == \
                (a0.LaborStatesNo, a0.aCount, len(a0.MgridBase), a0.AgentCount, self.econs[0].act_T, a0.shock_mode)
            if not same:
                raise ValueError("a batch shares LaborStatesNo, aCount, Mgrid size, AgentCount, act_T, shock_mode")
            if a.cycles != 0:
                raise NotImplementedError("only the infinite-horizon solve (cycles = 0, AH:237)")

    # ---- [HARK] Market.solve_agents over the active economies -------------------------
    def _solve_agents(self, active):
        arrays = []
        for k in active:
            a = self.agents[k]
            a.update()
            arrays.append(a.egm_arrays())
        cols = list(zip(*arrays))
        batch = EgmBatch.from_numpy(*(np.stack([np.asarray(x, dtype=np.float64) for x in col]) for col in cols[:7]),
                                    np.array(cols[7], dtype=np.float64), np.array(cols[8], dtype=np.float64),
                                    device=self.device)
        m, c, cycles, dist = egm_solve(batch, tol=self.agents[active[0]].tolerance, max_cycles=5000)
        for j, k in enumerate(active):
            a = self.agents[k]
            a.completed_cycles = int(cycles[j]) - 1
            a.solution_distance = float(dist[j])
            a.solution = [DeviceSolution(m[j], c[j], batch.M_grid[j], a.CRRA)]
        return batch, m, c

    # ---- [HARK] Market.make_history over the active economies -------------------------
    def _make_history(self, active, batch, m, c, ge_iter, rngs):
        n = len(active)
        econs = [self.econs[k] for k in active]
        agents = [self.agents[k] for k in active]
        N = agents[0].AgentCount
        act_T = econs[0].act_T
        for e in econs:
            e.reset()
        panel = BatchedPanel(n, N, act_T, device=self.device)
        lab_level = np.stack([sm.labor_levels(a.TauchenAux[0]) for a in agents])
        lab_cdf = np.stack([a.lab_cdf for a in agents])
        hist = np.stack([np.asarray(e.MrkvNow_hist[:act_T], dtype=np.int32) for e in econs])
        dev = lambda x: torch.as_tensor(np.ascontiguousarray(x)).to(self.device)  # noqa: E731
        panel.bind_models(m, c, batch.M_grid, dev(lab_level), dev(lab_cdf), dev(hist),
                          [e.market_constants() for e in econs])
        sow0 = [[e.sow_init["Mnow"], e.sow_init["Aprev"], e.sow_init["Mrkv"], e.sow_init["Rnow"], e.sow_init["Wnow"]]
                for e in econs]
        panel.reset(np.array([a.kInit for a in agents]),
                    np.stack([np.asarray(a.state_now["LaborSupplyState"]) for a in agents]), sow0)
        mode = agents[0].shock_mode
        if mode == "numpy":
            src = lambda nt: np.stack([rngs[k].random_sample((nt, N)) for k in active])  # noqa: E731
            panel.run(0, act_T, shock_mode="numpy", u_host_source=src, ge_iter=ge_iter)
        else:
            panel.run(0, act_T, shock_mode="philox", seeds=[a.shock_seed for a in agents], ge_iter=ge_iter)
        torch.cuda.synchronize(self.device)
        sow = panel.sow.cpu().numpy()
        a_now = panel.a.cpu().numpy()
        lab = panel.lab.cpu().numpy()
        hA = panel.hist_A.cpu().numpy()
        hM = panel.hist_M.cpu().numpy()
        for j, (e, a) in enumerate(zip(econs, agents)):
            s = dict(Mnow=float(sow[j, 0]), Aprev=float(sow[j, 1]), Mrkv=int(sow[j, 2]), Rnow=float(sow[j, 3]),
                     Wnow=float(sow[j, 4]))
            e.store_history(a, s, a_now[j].copy(), lab[j].copy(), hA[j].copy(), hM[j].copy())

    def solve(self):
        """[HARK] Market.solve for every economy; returns the per-economy GE iteration counts."""
        n = len(self.econs)
        rngs = [np.random.RandomState(a.shock_seed) for a in self.agents]
        old = [None] * n
        loops = [0] * n
        for e in self.econs:
            e.ge_log = []
        active = list(range(n))
        while active:
            ge_iter = loops[active[0]]
            batch, m, c = self._solve_agents(active)
            self._make_history(active, batch, m, c, ge_iter, rngs)
            still = []
            for k in active:
                e = self.econs[k]
                e._ge_iter = loops[k]
                new = e.update_dynamics()
                distance = new.distance(old[k]) if loops[k] > 0 else 1000000.0
                e.ge_log.append(dict(iter=loops[k], cycles=self.agents[k].completed_cycles + 1,
                                     intercept=list(e.intercept_prev), slope=list(e.slope_prev), distance=distance,
                                     Rnow=e.sow_state["Rnow"]))
                old[k] = new
                loops[k] += 1
                e.dynamics = new
                if distance >= e.tolerance and loops[k] < e.max_loops:
                    still.append(k)
            active = still
        return loops

    def results(self):
        """AH:257-258 per economy: r, saving rate, K/Y, K."""
        out = []
        for e in self.econs:
            K = float(np.mean(e.reap_state["aNow"][0]))
            d = e.DeprFac
            Y = e.sow_state["Mnow"] - (1 - d) * K
            out.append(dict(r=e.sow_state["Rnow"] - 1.0, saving_rate=d * K / Y, K_over_Y=K / Y, K=K,
                            ge_iters=len(e.ge_log), LaborAR=e.LaborAR, LaborSD=e.LaborSD, CRRA=e.CRRA))
        return out
