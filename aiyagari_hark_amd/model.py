"""Drop-in call surface of the reference: ``AiyagariType`` and
``AiyagariEconomy`` with the same constructor dictionaries, attributes and
solve/simulate hooks as ``Aiyagari_Support.py`` (AS), driven the way
``Aiyagari-HARK.py`` (AH:234-258) drives them:

    econ = AiyagariEconomy(**econ_dict); econ.verbose = False
    agent = AiyagariType(**agent_dict); agent.cycles = 0
    agent.get_economy_data(econ); econ.agents = [agent]
    econ.make_Mrkv_history(); econ.solve()
    econ.sow_state['Rnow'], econ.reap_state['aNow'][0], econ.sow_state['Mnow']
    agent.solution[0].cFunc[k].xInterpolators

HARK (econ-ark 0.12) is not available, so these classes do not subclass
``HARK.AgentType`` / ``HARK.Market``; they restate the parts of those base classes
the reference relies on (solve_agent's infinite-horizon loop, Market.solve /
make_history / update_dynamics) on top of libaiyagari.  Every per-grid-point and
per-agent computation runs in the HIP library; only O(S^2)-sized setup and the
once-per-GE-iteration regression run on the host.
"""
from __future__ import annotations

from copy import deepcopy

import numpy as np
import torch
from scipy import stats

from . import setup_math as sm
from .egm import EgmBatch, egm_solve, egm_step
from .interp import DeviceSolution
from .panel import DevicePanel

init_Aiyagari_agents = dict(LaborStatesNo=7, LaborAR=0.6, LaborSD=0.2, T_cycle=1, DiscFac=0.96, CRRA=1.0,
                            LbrInd=1.0, aMin=0.001, aMax=50.0, aCount=32, aNestFac=2,
                            MgridBase=sm.MGRID_BASE.copy(), AgentCount=140)          # AS:752-755

init_Aiyagari_economy = {                                                             # AS:1525-1551
    "verbose": True, "LaborStatesNo": 7, "LaborAR": 0.6, "LaborSD": 0.2, "act_T": 11000,
    "T_discard": 1000, "DampingFac": 0.5, "intercept_prev": [0.0, 0.0], "slope_prev": [1.0, 1.0],
    "DiscFac": 0.96, "CRRA": 1.0, "LbrInd": 1.0, "ProdB": 1.0, "ProdG": 1.0, "CapShare": 0.36,
    "DeprFac": 0.08, "DurMeanB": 8.0, "DurMeanG": 8.0, "SpellMeanB": 2.5, "SpellMeanG": 1.5,
    "UrateB": 0.0, "UrateG": 0.0, "RelProbBG": 0.75, "RelProbGB": 1.25, "MrkvNow_init": 0,
}


class AggregateSavingRule:
    """AS:1973-2005: A = exp(intercept + slope * log M)."""

    distance_criteria = ["slope", "intercept"]

    def __init__(self, intercept, slope):
        self.intercept = intercept
        self.slope = slope

    def __call__(self, Mnow):
        return np.exp(self.intercept + self.slope * np.log(Mnow))

    def distance(self, other):
        return max(float(abs(self.slope - other.slope)), float(abs(self.intercept - other.intercept)))


class AggShocksDynamicRule:
    """AS:2008-2020; distance = max over states of the rules' distances ([HARK] MetricObject)."""

    distance_criteria = ["AFunc"]

    def __init__(self, AFunc):
        self.AFunc = AFunc

    def distance(self, other):
        if len(self.AFunc) != len(other.AFunc):
            return float(abs(len(self.AFunc) - len(other.AFunc)))
        return max(a.distance(b) for a, b in zip(self.AFunc, other.AFunc))


class _Terminal:
    """update_solution_terminal (AS:892-904): cFunc = IdentityFunction(n_dims=2) for
    every discrete state.  Represented symbolically: the device EGM treats it as the
    cold-start guess c(m, M) = m."""

    def __init__(self, S, CRRA):
        self.S = S
        self.CRRA = CRRA


class AiyagariType:
    """AS:759-1415 on libaiyagari."""

    def __init__(self, device=None, shock_mode="numpy", shock_seed=0, panel_engine="auto", **kwds):
        params = init_Aiyagari_agents.copy()
        params.update(kwds)
        for k, v in params.items():
            setattr(self, k, v)
        self.params = params
        # [HARK] AgentType defaults used by the reference
        self.cycles = 1
        self.tolerance = 1e-6
        self.seed = 0
        self.verbose = getattr(self, "verbose", False)
        self.pseudo_terminal = False
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.shock_mode = shock_mode
        self.shock_seed = shock_seed
        self.panel_engine = panel_engine
        self.time_vary = []
        self.time_inv = ["DiscFac", "CRRA"]
        self.state_now = {"aNow": None, "mNow": None, "EmpNow": None, "LaborSupplyState": None}
        self.state_prev = dict(self.state_now)
        self.shock_vars = {"Mrkv": None}
        self.shocks = {}
        self.controls = {}
        self.solve_one_period = egm_step
        self.panel = None
        self.update()

    # ---- solve side -------------------------------------------------------------------
    def add_to_time_inv(self, *names):
        for n in names:
            if n not in self.time_inv:
                self.time_inv.append(n)

    def pre_solve(self):                      # AS:806-808
        self.update()
        self.precompute_arrays()

    def update(self):                         # AS:810-815
        self.make_grid()
        self.update_solution_terminal()

    def get_economy_data(self, Economy):      # AS:817-873
        self.T_sim = Economy.act_T
        self.kInit = Economy.KSS
        self.MrkvInit = Economy.sow_init["Mrkv"]
        self.Mgrid = Economy.MSS * np.asarray(self.MgridBase)
        self.AFunc = Economy.AFunc
        for name in ("DeprFac", "CapShare", "LbrInd", "UrateB", "UrateG", "ProdB", "ProdG", "MrkvIndArray",
                     "MrkvEmplArray", "TauchenAux"):
            setattr(self, name, getattr(Economy, name))
        self.MrkvAggArray = Economy.MrkvArray
        self.add_to_time_inv("Mgrid", "AFunc", "DeprFac", "CapShare", "LaborStatesNo", "LaborAR", "LaborSD",
                             "UrateB", "LbrInd", "UrateG", "ProdB", "ProdG", "MrkvIndArray", "MrkvAggArray",
                             "MrkvEmplArray", "TauchenAux")

    def make_grid(self):                      # AS:875-890
        self.aGrid = sm.make_grid_exp_mult(self.aMin, self.aMax, self.aCount, self.aNestFac)
        self.add_to_time_inv("aGrid")
        self.TauchenAux = sm.labor_tauchen(self.LaborStatesNo, self.LaborAR, self.LaborSD)
        self.add_to_time_inv("TauchenAux")

    def update_solution_terminal(self):       # AS:892-904
        self.solution_terminal = _Terminal(4 * self.LaborStatesNo, self.CRRA)

    def precompute_arrays(self):              # AS:906-1037
        # Krusell-Smith mode (UrateB/UrateG > 0) needs nothing more here: the reference's
        # household solve keeps LSStates as next-period labour income in the unemployed
        # sub-states too (AS:990-1018), and L = (1 - Urate) LbrInd enters next_prices.
        self.egm_batch = EgmBatch.from_numpy(*self.egm_arrays(), device=self.device)
        self.add_to_time_inv("egm_batch")

    def egm_arrays(self):
        """Host inputs of solve_Aiyagari for the current AFunc: (aGrid, Mgrid, P, R_next,
        W_next, M_next, lab, DiscFac, CRRA), precompute_arrays (AS:906-1037) reduced to
        its unique [n_M, S] content."""
        S = 4 * self.LaborStatesNo
        R, W, M = sm.next_prices([f.intercept for f in self.AFunc], [f.slope for f in self.AFunc], self.Mgrid, S,
                                 self.UrateB, self.UrateG, self.LbrInd, self.ProdB, self.ProdG, self.CapShare,
                                 self.DeprFac)
        self.LSStates = sm.labor_levels(self.TauchenAux[0])
        lab = np.array([self.LSStates[sp // 4] for sp in range(S)])
        return self.aGrid, self.Mgrid, self.MrkvIndArray, R, W, M, lab, self.DiscFac, self.CRRA

    def solve(self, verbose=False):
        """[HARK] AgentType.solve -> solve_agent (cycles = 0: infinite horizon)."""
        if self.cycles != 0:
            raise NotImplementedError("only the infinite-horizon solve (cycles = 0, AH:237) is on the hot path")
        self.pre_solve()
        m, c, cycles, dist = egm_solve(self.egm_batch, tol=self.tolerance, max_cycles=5000)
        self.completed_cycles = int(cycles[0]) - 1
        self.solution_distance = float(dist[0])
        self.solution = [DeviceSolution(m[0], c[0], self.egm_batch.M_grid[0], self.CRRA)]
        self.post_solve()
        return self.solution

    def post_solve(self):
        pass

    def save_solution(self, path, economy=None):
        """Policies plus the agent's AFunc to ``.npz``.  With
        ``economy`` the file also records how many GE iterations it has completed, so a
        later ``load_solution(path, economy=...)`` can resume ``economy.solve()``."""
        extra = {}
        if economy is not None:
            extra["ge_iterations"] = np.int64(getattr(economy, "ge_iterations_done", 0))
        self.solution[0].save(path, AFunc=self.AFunc, **extra)

    def load_solution(self, path, economy=None):
        """Restore ``solution[0]`` (device-resident) and AFunc written by ``save_solution``.

        With ``economy`` the saved saving rules also become the economy's state, so that
        ``economy.solve()`` resumes the fixed point instead of mixing two rules: its AFunc
        and the damping state ``intercept_prev`` / ``slope_prev`` that calc_AFunc damps
        against (AS:1950-1951; updated in place, the reference's aliasing quirk Q9), and
        the GE iteration count keying the Philox shock counter.  Without ``economy`` the
        loaded solution is for evaluation (``cFunc``) and for simulation only."""
        sol, afunc, meta = DeviceSolution.load(path, self.device, with_meta=True)
        self.solution = [sol]
        if afunc is not None:
            self.AFunc = [AggregateSavingRule(float(i), float(s)) for i, s in afunc]
            if economy is not None:
                economy.intercept_prev[:] = [float(i) for i, _ in afunc]
                economy.slope_prev[:] = [float(s) for _, s in afunc]
                economy.AFunc = [AggregateSavingRule(float(i), float(s)) for i, s in afunc]
        if economy is not None:
            economy.ge_iter_base = int(meta.get("ge_iterations", 0))
            economy.ge_iterations_done = economy.ge_iter_base
        return self.solution

    # ---- simulation side ---------------------------------------------------------------
    def reset(self):                          # AS:1158
        self.initialize_sim()

    @property
    def ks_mode(self):
        """Krusell-Smith employment (UrateB or UrateG > 0): exact-count employment
        transitions each period (AS:1222-1240) and the unemployed sub-states' policies."""
        return self.UrateB != 0.0 or self.UrateG != 0.0

    def initialize_sim(self):                 # AS:1164-1171 + [HARK] AgentType.initialize_sim
        self.shocks["Mrkv"] = self.MrkvInit
        emp, lab, self.RNG = sm.birth_states(self.AgentCount, self.LaborStatesNo, self.UrateB, seed=self.seed,
                                             Mrkv=int(self.MrkvInit), UrateG=self.UrateG, with_rng=True)
        self.state_now["EmpNow"] = emp
        self.state_now["LaborSupplyState"] = lab
        self._emp_host = emp
        # make_emp_idx_arrays (AS:1171); the agent RNG above continues into the per-period
        # employment permutations (the panel's employment is drawn on the host, exactly)
        self.emp_trans = sm.employment_transitions(self.AgentCount, self.UrateB, self.UrateG, self.MrkvEmplArray,
                                                   self.MrkvAggArray) if self.ks_mode else None
        self.t_sim = 0
        if self.panel is None or self.panel.n_local != self.AgentCount or self.panel.act_T != self.T_sim \
                or self.panel.engine != self.panel_engine:
            self.panel = DevicePanel(self.AgentCount, device=self.device, act_T=self.T_sim, engine=self.panel_engine)
        self.lab_cdf = sm.choice_cdf_table(self.TauchenAux[1])          # agent's own chain (AS:1245, Q5)
        self.state_now["aNow"] = np.full(self.AgentCount, float(self.kInit))   # sim_birth (AS:1213)
        self._hook_const = None

    # ---- per-period hooks ([HARK] AgentType.simulate / sim_one_period, AS:1161, 1217-1415) ----
    # One libaiyagari launch per hook over device-resident agent states: the surface a
    # driver stepping Market.make_history period by period (sow -> cultivate -> reap ->
    # mill -> store) calls.  AiyagariEconomy.make_history(engine="fused") runs the same
    # periods as one fused pass; the two agree bit for bit on labour draws.
    def market_action(self):                  # AS:1161
        self.simulate(1)

    def simulate(self, sim_periods=1):        # [HARK] AgentType.simulate
        for _ in range(int(sim_periods)):
            self.sim_one_period()

    def sim_one_period(self):                 # [HARK] AgentType.sim_one_period (no death)
        self._to_device()
        for var in self.state_now:
            self.state_prev[var] = self.state_now[var]
        self.get_shocks()
        self.get_states()
        self.get_controls()
        self.get_poststates()
        self.t_sim += 1

    def _to_device(self):
        """Agent states as device arrays (a: float64, LaborSupplyState / EmpNow: uint8)
        plus the hooks' constant tables, made once per simulated history."""
        st, dev, N = self.state_now, self.device, self.AgentCount
        for k, dt in (("aNow", torch.float64), ("LaborSupplyState", torch.uint8), ("EmpNow", torch.uint8)):
            if not torch.is_tensor(st[k]):
                st[k] = torch.as_tensor(np.asarray(st[k]).astype(np.float64 if dt == torch.float64 else np.uint8)
                                        ).to(dev)
            if st[k].numel() != N:
                raise ValueError(f"state {k} holds {st[k].numel()} agents, AgentCount = {N}")
        if self._hook_const is None:
            from . import _lib
            lvl = sm.labor_levels(self.TauchenAux[0])
            self._hook_const = dict(
                h=_lib.handle(dev.index if dev.index is not None else torch.cuda.current_device()),
                lvl=torch.as_tensor(lvl, dtype=torch.float64).to(dev),
                cdf=torch.as_tensor(self.lab_cdf, dtype=torch.float64).to(dev),
                n_lab=int(self.lab_cdf.shape[0]))

    def employment_next(self, mrkv_now):
        """This period's employment (get_shocks, AS:1222-1240) from the last one, host-side
        with the agent RNG; everyone stays employed outside Krusell-Smith mode."""
        if self.ks_mode:
            self._emp_host = sm.employment_step(self._emp_host, mrkv_now, self.UrateB, self.emp_trans, self.RNG)
        return self._emp_host

    def get_shocks(self):                     # AS:1217-1256
        from . import _lib
        k = self._hook_const
        if self.ks_mode:
            emp = self.employment_next(self.shocks["Mrkv"])
            self.state_now["EmpNow"] = torch.as_tensor(emp.astype(np.uint8)).to(self.device)
        else:
            self.state_now["EmpNow"] = self.state_prev["EmpNow"]
        lab = self.state_prev["LaborSupplyState"].clone()
        u = None
        if self.shock_mode == "numpy":   # np.random.choice per agent on the global RNG (AS:1254)
            u = torch.as_tensor(np.random.random_sample(self.AgentCount)).to(self.device)
        elif self.shock_mode != "philox":
            raise ValueError(f"shock_mode {self.shock_mode!r}")
        s = _lib.stream_ptr()
        k["h"].check(k["h"].lib.aiy_get_shocks(k["h"].h, k["n_lab"], _lib.ptr(k["cdf"]), self.AgentCount, 0,
                                               _lib.ptr(lab), _lib.ptr(u), int(self.shock_seed) & ((1 << 64) - 1),
                                               int(getattr(self, "ge_iter", 0)), int(self.t_sim), s), "aiy_get_shocks")
        self.state_now["LaborSupplyState"] = lab

    def get_states(self):                     # AS:1259-1283
        from . import _lib
        k = self._hook_const
        m = torch.empty(self.AgentCount, dtype=torch.float64, device=self.device)
        k["h"].check(k["h"].lib.aiy_get_states(k["h"].h, _lib.ptr(k["lvl"]), self.AgentCount, float(self.Rnow),
                                               float(self.Wnow), _lib.ptr(self.state_prev["aNow"]),
                                               _lib.ptr(self.state_now["LaborSupplyState"]),
                                               _lib.ptr(self.state_now["EmpNow"]), _lib.ptr(m), _lib.stream_ptr()),
                     "aiy_get_states")
        self.state_now["mNow"] = m

    def get_controls(self):                   # AS:1286-1408
        from . import _lib
        k = self._hook_const
        sol = self.solution[0]
        S, n_M, n1 = sol.m_tab.shape
        Mg = np.ascontiguousarray(sol.M_grid_host(), dtype=np.float64)
        c = torch.empty(self.AgentCount, dtype=torch.float64, device=self.device)
        k["h"].check(k["h"].lib.aiy_get_controls(k["h"].h, S, n_M, n1 - 1, _lib.ptr(sol.m_tab), _lib.ptr(sol.c_tab),
                                                 Mg.ctypes.data_as(_lib.c_double_p), int(self.shocks["Mrkv"]),
                                                 float(self.Mnow), self.AgentCount, _lib.ptr(self.state_now["mNow"]),
                                                 _lib.ptr(self.state_now["LaborSupplyState"]),
                                                 _lib.ptr(self.state_now["EmpNow"]), _lib.ptr(c), _lib.stream_ptr()),
                     "aiy_get_controls")
        self.controls["cNow"] = c

    def get_poststates(self):                 # AS:1411-1415
        from . import _lib
        k = self._hook_const
        a = torch.empty(self.AgentCount, dtype=torch.float64, device=self.device)
        k["h"].check(k["h"].lib.aiy_get_poststates(k["h"].h, self.AgentCount, _lib.ptr(self.state_now["mNow"]),
                                                   _lib.ptr(self.controls["cNow"]), _lib.ptr(a), _lib.stream_ptr()),
                     "aiy_get_poststates")
        self.state_now["aNow"] = a


class AiyagariEconomy:
    """AS:1555-1964 on libaiyagari (Market restated)."""

    def __init__(self, agents=None, tolerance=0.01, **kwds):
        agents = agents if agents is not None else list()
        params = deepcopy(init_Aiyagari_economy)
        params.update(kwds)          # keeps the caller's intercept_prev/slope_prev lists (quirk Q9)
        self.agents = agents
        self.tolerance = tolerance
        self.max_loops = 1000
        self.sow_vars = ["Mnow", "Aprev", "Mrkv", "Rnow", "Wnow"]
        self.reap_vars = ["aNow", "EmpNow"]
        self.track_vars = ["Mrkv", "Aprev", "Mnow", "Urate"]
        self.dyn_vars = ["AFunc"]
        for k, v in params.items():
            setattr(self, k, v)
        self.sow_init = {v: None for v in self.sow_vars}
        self.sow_state = {v: None for v in self.sow_vars}
        self.reap_state = {v: [] for v in self.reap_vars}
        self.history = {v: [] for v in self.track_vars}
        self.update()

    def update(self):                         # AS:1593-1629
        self.AFunc = [AggregateSavingRule(self.intercept_prev[j], self.slope_prev[j]) for j in range(2)]
        ss = sm.steady_state(self.CRRA, self.DiscFac, self.DeprFac, self.CapShare, self.LbrInd)
        for k, v in ss.items():
            setattr(self, k, v)
        self.convertKtoY = lambda KtoY: KtoY ** (1.0 / (1.0 - self.CapShare))
        self.rFunc = lambda k: self.CapShare * k ** (self.CapShare - 1.0)
        self.Wfunc = lambda k: ((1.0 - self.CapShare) * k ** (self.CapShare))
        self.sow_init.update(KtoLnow=self.KtoLSS, Mnow=self.MSS, Aprev=self.KSS, Rnow=self.RSS, Wnow=self.WSS, Mrkv=0)
        self.make_MrkvArray()

    def make_MrkvArray(self):                 # AS:1639-1791
        agg, E = sm.employment_chain(self.DurMeanB, self.DurMeanG, self.SpellMeanB, self.SpellMeanG, self.UrateB,
                                     self.UrateG, self.RelProbBG, self.RelProbGB)
        T = sm.labor_tauchen(self.LaborStatesNo, self.LaborAR, self.LaborSD)
        self.MrkvArray = agg
        self.MrkvEmplArray = E
        self.MrkvIndArray = sm.kron_states(T[1], E)
        self.TauchenAux = T

    def make_Mrkv_history(self):              # AS:1793-1805
        self.MrkvNow_hist = sm.markov_history(self.MrkvArray, self.act_T, self.MrkvNow_init, seed=0)

    def reset(self):                          # AS:1631-1637 + [HARK] Market.reset
        self.Shk_idx = 0
        self.history = {v: [] for v in self.track_vars}
        for v in self.sow_state:
            self.sow_state[v] = self.sow_init[v]
        for a in self.agents:
            a.reset()

    # ---- GE fixed point ----------------------------------------------------------------
    def solve_agents(self):
        for a in self.agents:
            a.solve()

    def make_history(self):
        """[HARK] Market.make_history: act_T periods of sow -> cultivate -> reap -> mill ->
        store.  history_engine "fused" (default): all periods on device in one pass
        (libaiyagari aiy_sim_periods); "hooks": the period loop on the host calling the
        market and agent hooks one at a time (aiy_get_shocks .. aiy_sum per period)."""
        if len(self.agents) != 1:
            raise NotImplementedError("the reference economy has exactly one AgentType")
        if getattr(self, "history_engine", "fused") == "hooks":
            return self.make_history_hooks()
        agent = self.agents[0]
        self.reset()
        p = agent.panel
        sol = agent.solution[0]
        lab_level = torch.as_tensor(agent.LSStates if hasattr(agent, "LSStates") else
                                    sm.labor_levels(agent.TauchenAux[0]), dtype=torch.float64).to(agent.device)
        lab_cdf = torch.as_tensor(agent.lab_cdf, dtype=torch.float64).to(agent.device)
        hist = torch.as_tensor(np.asarray(self.MrkvNow_hist, dtype=np.int32)).to(agent.device)
        market = self.market_constants()
        ks = agent.ks_mode
        p.bind_model(sol.m_tab, sol.c_tab, sol.M_grid, lab_level, lab_cdf, hist, market, unemployed=ks)
        p.reset(agent.kInit, agent.state_now["LaborSupplyState"], self.sow_init["Mnow"], self.sow_init["Aprev"],
                self.sow_init["Mrkv"], self.sow_init["Rnow"], self.sow_init["Wnow"])
        ge_iter = getattr(self, "_ge_iter", 0)
        N = agent.AgentCount
        urate = []
        emp_src = None
        if ks:
            mrkv = np.asarray(self.MrkvNow_hist)
            clock = [0]

            def emp_src(n):   # EmpNow of the next n periods; the period's Mrkv is the sown one
                out = np.empty((n, N), dtype=np.uint8)
                for k in range(n):
                    t = clock[0]
                    now = self.sow_init["Mrkv"] if t == 0 else mrkv[t - 1]
                    e = agent.employment_next(now)
                    out[k] = e
                    urate.append(1.0 - float(np.mean(e)))          # AS:1873 (recorded only)
                    clock[0] = t + 1
                return out
        if agent.shock_mode == "numpy":
            src = lambda n: np.random.random_sample((n, N))  # noqa: E731 -- the reference's global RNG
            p.run(0, self.act_T, shock_mode="numpy", u_host_source=src, ge_iter=ge_iter, emp_source=emp_src)
        else:
            p.run(0, self.act_T, shock_mode="philox", seed=agent.shock_seed, ge_iter=ge_iter, emp_source=emp_src)
        torch.cuda.synchronize(agent.device)
        self.store_history(agent, p.sow_host(), p.a.cpu().numpy(), p.lab.cpu().numpy(), p.hist_A.cpu().numpy(),
                           p.hist_M.cpu().numpy(), agent._emp_host if ks else None, urate if ks else None)

    # ---- [HARK] Market's per-period hooks ----------------------------------------------
    def make_history_hooks(self):
        self.reset()
        for a in self.agents:
            a.ge_iter = getattr(self, "_ge_iter", 0)
        for _ in range(self.act_T):
            self.sow()
            self.cultivate()
            self.reap()
            self.mill()
            self.store()
        self.history = {k: np.asarray(v) for k, v in self.history.items()}
        self.reap_state = {k: [x.cpu().numpy().astype(np.float64) if torch.is_tensor(x) else x for x in v]
                           for k, v in self.reap_state.items()}

    def sow(self):                           # [HARK] Market.sow
        for var in self.sow_vars:
            for a in self.agents:
                if var in a.shock_vars:
                    a.shocks[var] = self.sow_state[var]
                else:
                    setattr(a, var, self.sow_state[var])

    def cultivate(self):                      # [HARK] Market.cultivate
        for a in self.agents:
            a.market_action()

    def reap(self):                           # [HARK] Market.reap
        for var in self.reap_vars:
            self.reap_state[var] = [a.state_now[var] for a in self.agents]

    def mill(self):                           # [HARK] Market.mill
        product = self.mill_rule(**self.reap_state)
        for i, var in enumerate(self.sow_vars):
            self.sow_state[var] = product[i]

    def store(self):                          # [HARK] Market.store
        for var in self.track_vars:
            if var in self.sow_state:
                v = self.sow_state[var]
            elif var in self.reap_state:
                v = self.reap_state[var]
            else:
                v = getattr(self, var)
            self.history[var].append(v)

    def market_constants(self):
        """Constants of calc_R_and_W (AS:1867-1894) for the device mill."""
        return dict(CapShare=self.CapShare, DeprFac=self.DeprFac, prod=(self.ProdB, self.ProdG),
                    agg_L=((1.0 - self.UrateB) * self.LbrInd, (1.0 - self.UrateG) * self.LbrInd))

    def store_history(self, agent, sow, aNow, lab, hist_A, hist_M, emp=None, urate=None):
        """Write back one simulated history the way [HARK] Market.make_history leaves it."""
        self.Shk_idx = self.act_T
        for v in self.sow_vars:
            self.sow_state[v] = sow[v]
        emp = np.ones(agent.AgentCount) if emp is None else np.asarray(emp, dtype=np.float64)
        self.reap_state = {"aNow": [aNow], "EmpNow": [emp]}
        agent.state_now["aNow"] = aNow
        agent.state_now["LaborSupplyState"] = lab.astype(np.int64)
        agent.state_now["EmpNow"] = emp.astype(bool)
        self.Urate = 1.0 - float(np.mean(emp))
        self.history = {"Mrkv": list(np.asarray(self.MrkvNow_hist[:self.act_T])), "Aprev": hist_A, "Mnow": hist_M,
                        "Urate": np.zeros(self.act_T) if urate is None else np.asarray(urate)}

    def update_dynamics(self):                # [HARK] Market.update_dynamics
        dyn = self.calc_dynamics(Mnow=self.history["Mnow"], Aprev=self.history["Aprev"])
        for v in self.dyn_vars:
            for a in self.agents:
                setattr(a, v, getattr(dyn, v))
        return dyn

    def solve(self):                          # [HARK] Market.solve
        go = True
        loops = 0
        old = None
        self.ge_log = []
        base = int(getattr(self, "ge_iter_base", 0))   # > 0 when resuming from load_solution
        while go:
            self._ge_iter = base + loops                 # keys the Philox shock counter
            self.solve_agents()
            self.make_history()
            new = self.update_dynamics()
            distance = new.distance(old) if loops > 0 else 1000000.0
            self.ge_log.append(dict(iter=loops, cycles=self.agents[0].completed_cycles + 1,
                                    intercept=list(self.intercept_prev), slope=list(self.slope_prev),
                                    distance=distance, Rnow=self.sow_state["Rnow"]))
            old = new
            loops += 1
            self.ge_iterations_done = base + loops
            go = distance >= self.tolerance and loops < self.max_loops
        self.dynamics = new

    # ---- market hooks (AS:1808-1964) ---------------------------------------------------
    def mill_rule(self, aNow, EmpNow):
        return self.calc_R_and_W(aNow, EmpNow)

    def calc_dynamics(self, Mnow, Aprev):
        return self.calc_AFunc(Mnow, Aprev)

    def calc_R_and_W(self, aNow, EmpNow):
        """AS:1839-1894 for one period given the agents' assets (scalar formulas; the
        device path fuses this into aiy_sim_periods).  Device-resident harvests (the
        per-period hooks) are averaged on device (aiy_sum)."""
        if torch.is_tensor(aNow[0]):
            Aprev = self._device_mean(aNow)
            Urate = 1.0 - self._device_mean([e.to(torch.float64) for e in EmpNow])
        else:
            Aprev = float(np.mean(np.array(aNow)))
            Urate = 1.0 - float(np.mean(np.array(EmpNow)))
        self.Urate = Urate
        Mrkv = self.MrkvNow_hist[self.Shk_idx]
        Prod, L = (self.ProdB, (1.0 - self.UrateB) * self.LbrInd) if Mrkv == 0 else \
            (self.ProdG, (1.0 - self.UrateG) * self.LbrInd)
        self.Shk_idx += 1
        k = Aprev / L
        R = 1.0 + Prod * self.rFunc(k) - self.DeprFac
        W = Prod * self.Wfunc(k)
        self.KtoLnow = k
        return R * Aprev + W * L, Aprev, Mrkv, R, W

    @staticmethod
    def _device_mean(xs):
        """np.mean(np.array(xs)) of device arrays: fixed-order sums (aiy_sum), one
        host read."""
        from . import _lib
        out = torch.empty(len(xs), dtype=torch.float64, device=xs[0].device)
        h = _lib.handle(xs[0].device.index)
        for i, x in enumerate(xs):
            h.check(h.lib.aiy_sum(h.h, _lib.ptr(x), x.numel(), _lib.ptr(out[i:i + 1]), _lib.stream_ptr()), "aiy_sum")
        return float(out.cpu().numpy().sum()) / sum(x.numel() for x in xs)

    def calc_AFunc(self, Mnow, Aprev):
        """AS:1896-1964: per-state OLS of log A_t on log M_{t-1} after T_discard, damped."""
        T = len(Mnow)
        d = self.T_discard
        w = 1.0 - self.DampingFac
        logA = np.log(np.asarray(Aprev)[d:T])
        logM = np.log(np.asarray(Mnow)[d - 1:T - 1])
        hist = np.asarray(self.MrkvNow_hist)[d - 1:T - 1]
        rules, rsq = [], []
        for i in range(self.MrkvArray.shape[0]):
            these = i == hist
            res = stats.linregress(logM[these], logA[these])
            intercept = w * res.intercept + (1.0 - w) * self.intercept_prev[i]
            slope = w * res.slope + (1.0 - w) * self.slope_prev[i]
            rules.append(AggregateSavingRule(intercept, slope))
            rsq.append(res.rvalue ** 2)
            self.intercept_prev[i] = intercept
            self.slope_prev[i] = slope
        if self.verbose:
            print("intercept=" + str(self.intercept_prev) + ", slope=" + str(self.slope_prev) + ", r-sq=" + str(rsq))
        return AggShocksDynamicRule(rules)
