"""Device panel through the libaiyagari C ABI.

A ``DevicePanel`` owns the agents of one rank (assets, labour states), the device
market state ("sow_state") and the per-period history buffers.  ``run`` enqueues
whole blocks of periods; the host never touches per-agent data inside a history.

Shock sources (``u`` of get_shocks, Aiyagari_Support.py:1253-1254):
  * ``"numpy"``  -- uniforms drawn on the host from NumPy's *global* RandomState in
    exactly the order the reference's ``np.random.choice`` calls consume them
    (agent-major per period, periods in order); seeding ``np.random.seed(k)``
    before a solve makes the GPU history reproduce the reference's.
  * ``"philox"`` -- counter-based Philox4x32-10 on device (key = seed, counter =
    (GE iteration << 20 | t, global agent index)); independent of sharding.

Two engines run the same per-period semantics:
  * ``"grid"``  -- one launch per period over the whole population (aiy_sim_periods);
    the engine for large panels (configs[1], configs[3]) and the only sharded one.
  * ``"block"`` -- one workgroup per calibration with the agents resident in LDS for a
    whole block of periods (aiy_sim_block_periods); the engine for the reference's own
    350-700-agent panels, where a launch per period would be launch-bound.
``"auto"`` picks ``block`` for unsharded panels of at most aiy_sim_block_max_agents().
``BatchedPanel`` runs many calibrations' panels in one launch (Table II sweep).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

F64 = torch.float64


class DevicePanel:
    def __init__(self, n_local: int, device=None, agent_offset: int = 0, n_total: int | None = None,
                 act_T: int = 11000, engine: str = "auto"):
        self.device = torch.device(device or "cuda")
        if engine not in ("auto", "grid", "block"):
            raise ValueError(f"engine {engine!r}")
        self.n_local = int(n_local)
        self.agent_offset = int(agent_offset)
        self.n_total = int(n_total if n_total is not None else n_local)
        self.a = torch.empty(self.n_local, dtype=F64, device=self.device)
        self.lab = torch.empty(self.n_local, dtype=torch.uint8, device=self.device)
        self.sow = torch.zeros(_lib.AIY_SOW_DOUBLES, dtype=F64, device=self.device)
        self.act_T = int(act_T)
        self.hist_A = torch.zeros(self.act_T, dtype=F64, device=self.device)
        self.hist_M = torch.zeros(self.act_T, dtype=F64, device=self.device)
        self._model = None
        self.engine = engine

    def _engine(self, h):
        if self.engine != "auto":
            return self.engine
        small = self.n_local <= h.lib.aiy_sim_block_max_agents()
        return "block" if small and self.n_total == self.n_local and self.agent_offset == 0 else "grid"

    def reset(self, a0, lab0, Mnow, Aprev, Mrkv, Rnow, Wnow):
        """sim_birth + Market.reset sow_init (Aiyagari_Support.py:1621-1628)."""
        a0 = np.broadcast_to(np.asarray(a0, dtype=np.float64), (self.n_local,))
        self.a.copy_(torch.from_numpy(np.array(a0, dtype=np.float64, order="C")))
        self.lab.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(lab0, dtype=np.uint8))))
        sow = np.zeros(_lib.AIY_SOW_DOUBLES)
        sow[:6] = [Mnow, Aprev, Mrkv, Rnow, Wnow, 0.0]
        self.sow.copy_(torch.from_numpy(sow))
        self.hist_A.zero_()
        self.hist_M.zero_()

    def bind_model(self, m_pol, c_pol, M_grid, lab_level, lab_cdf, mrkv_hist, market: dict, unemployed=False):
        """unemployed: build the policy tables of the unemployed sub-states too (Krusell-Smith
        mode: run(..., emp_source=...))."""
        S, n_M, n1 = m_pol.shape
        n_lab = int(lab_level.numel())
        keep = dict(M_grid=M_grid.contiguous(), lab_level=lab_level.contiguous(), lab_cdf=lab_cdf.contiguous(),
                    mrkv_hist=mrkv_hist.to(torch.int32).contiguous())
        # merged policy tables (aiy_panel_build, once per history)
        h = _lib.handle(self.device.index)
        keep["tables"] = build_tables(h, m_pol[None], c_pol[None], n_lab, self.device, unemployed)
        ptrs = [_lib.ptr(keep[k]) for k in ("tables", "M_grid", "lab_level", "lab_cdf", "mrkv_hist")]
        # periods a call may simulate: the history buffers and the Mrkv history must cover them
        self.model_T = min(self.act_T, int(keep["mrkv_hist"].numel()))
        pm = _lib.PanelModel(S, n_M, n1 - 1, n_lab, *ptrs, self.model_T, int(bool(unemployed)))
        mk = make_market(market)
        pb = _lib.PanelBatch(1, S, n_M, n1 - 1, n_lab, *ptrs, int(bool(unemployed)))
        self._model = (pm, mk, keep, pb)

    def run(self, t0: int, n_periods: int, shock_mode="philox", seed=0, ge_iter=0, u_host_source=None,
            chunk=1000, stream=None, allreduce=None, emp_source=None):
        """Simulate periods [t0, t0 + n_periods).  For shock_mode='numpy', u_host_source(n)
        must return the next n x n_local uniforms (host).

        emp_source: Krusell-Smith mode (bind_model(unemployed=True)): emp_source(n) returns
        the employment states (0/1) of the next n periods, [n, n_local] (host); None:
        everyone employed.

        allreduce: for an agent-sharded panel without a communicator bound in the library
        (parallel.bind_rccl), a callable that sums the 1-element device tensor it is given
        over all ranks in place (parallel.torch_allreduce: torch.distributed over RCCL or
        gloo); each period then runs as aiy_sim_period_local -> allreduce ->
        aiy_sim_period_prices."""
        if self._model is None:
            raise RuntimeError("bind_model() first")
        if t0 < 0 or n_periods < 0 or t0 + n_periods > self.model_T:
            raise ValueError(f"periods [{t0}, {t0 + n_periods}) outside the history [0, {self.model_T})")
        if shock_mode not in ("philox", "numpy"):
            raise ValueError(shock_mode)
        pm, mk, _, pb = self._model
        if emp_source is not None and not pm.unemployed:
            raise ValueError("employment states need bind_model(..., unemployed=True)")
        h = _lib.handle(self.device.index)
        sp = _lib.stream_ptr(stream)
        if allreduce is not None:
            self._run_stepwise(h, pm, mk, t0, n_periods, shock_mode, seed, ge_iter, u_host_source, chunk, sp,
                               allreduce, emp_source, stream)
            return
        if self._engine(h) == "block":
            if self.n_total != self.n_local or self.agent_offset != 0:
                raise ValueError("the block engine does not shard agents")
            seeds = (ctypes.c_uint64 * 1)(int(seed) & ((1 << 64) - 1))
            run_block(h, pb, ctypes.byref(mk), self.n_local, self.a, self.lab, seeds, ge_iter, t0, n_periods,
                      self.act_T, self.sow, self.hist_A, self.hist_M, shock_mode, u_host_source, chunk, sp, stream,
                      emp_source)
            return
        if shock_mode == "philox" and emp_source is None:
            h.check(h.lib.aiy_sim_periods(h.h, ctypes.byref(pm), ctypes.byref(mk), self.n_local, self.agent_offset,
                                          self.n_total, _lib.ptr(self.a), _lib.ptr(self.lab), None, 0, None, 0,
                                          int(seed) & ((1 << 64) - 1), int(ge_iter), int(t0), int(n_periods),
                                          _lib.ptr(self.sow), _lib.ptr(self.hist_A), _lib.ptr(self.hist_M), sp),
                    "aiy_sim_periods")
            return
        t = t0
        end = t0 + n_periods
        while t < end:
            n = min(chunk, end - t)
            ud = _host_block(u_host_source, n, (n, self.n_local), np.float64, self.device) \
                if shock_mode == "numpy" else None
            ed = _host_block(emp_source, n, (n, self.n_local), np.uint8, self.device) if emp_source else None
            h.check(h.lib.aiy_sim_periods(h.h, ctypes.byref(pm), ctypes.byref(mk), self.n_local, self.agent_offset,
                                          self.n_total, _lib.ptr(self.a), _lib.ptr(self.lab), _lib.ptr(ud),
                                          self.n_local, _lib.ptr(ed), self.n_local, int(seed) & ((1 << 64) - 1),
                                          int(ge_iter), int(t), int(n), _lib.ptr(self.sow),
                                          _lib.ptr(self.hist_A), _lib.ptr(self.hist_M), sp), "aiy_sim_periods")
            torch.cuda.current_stream(self.device).synchronize() if stream is None else stream.synchronize()
            del ud, ed
            t += n

    def _run_stepwise(self, h, pm, mk, t0, n_periods, shock_mode, seed, ge_iter, u_host_source, chunk, sp,
                      allreduce, emp_source=None, stream=None):
        """Sharded periods with the all-reduce done by the caller between the library's two
        steps (Aiyagari_Support.py:1868, np.mean over all ranks' agents)."""
        red = self.sow[6:7]
        # the all-reduce runs on the stream the library steps were enqueued on (the nccl
        # backend enqueues on torch's current stream, the gloo path syncs it before its copy)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        t, end = t0, t0 + n_periods
        while t < end:
            n = min(chunk, end - t)
            ud = _host_block(u_host_source, n, (n, self.n_local), np.float64, self.device) \
                if shock_mode == "numpy" else None
            ed = _host_block(emp_source, n, (n, self.n_local), np.uint8, self.device) if emp_source else None
            for k in range(n):
                up = None if ud is None else ud[k].data_ptr()
                ep = None if ed is None else ed[k].data_ptr()
                h.check(h.lib.aiy_sim_period_local(h.h, ctypes.byref(pm), self.n_local, self.agent_offset,
                                                   _lib.ptr(self.a), _lib.ptr(self.lab), up, ep,
                                                   int(seed) & ((1 << 64) - 1), int(ge_iter), int(t + k),
                                                   _lib.ptr(self.sow), sp), "aiy_sim_period_local")
                with torch.cuda.stream(st):
                    allreduce(red)
                h.check(h.lib.aiy_sim_period_prices(h.h, ctypes.byref(pm), ctypes.byref(mk), self.n_total, int(t + k),
                                                    _lib.ptr(self.sow), _lib.ptr(self.hist_A), _lib.ptr(self.hist_M),
                                                    sp), "aiy_sim_period_prices")
            if ud is not None or ed is not None:
                st.synchronize()
            del ud, ed
            t += n

    def sow_host(self):
        s = self.sow.cpu().numpy()
        return dict(Mnow=float(s[0]), Aprev=float(s[1]), Mrkv=int(s[2]), Rnow=float(s[3]), Wnow=float(s[4]),
                    Urate=float(s[5]))


def _host_block(source, n, shape, dtype, device):
    """The next n periods of a host-side source (uniforms / employment) as a device tensor
    of `shape` (one calibration) or [n_cal, *shape] (batched)."""
    x = np.ascontiguousarray(source(n), dtype=dtype)
    if x.shape != shape:
        raise ValueError(f"host block shape {x.shape} != {shape}")
    return torch.from_numpy(x).to(device)


def make_market(market: dict) -> "_lib.Market":
    return _lib.Market(market["CapShare"], market["DeprFac"], (ctypes.c_double * 2)(*market["prod"]),
                       (ctypes.c_double * 2)(*market["agg_L"]))


def build_tables(h, m_pol, c_pol, n_lab, device, unemployed=False):
    """Merged policy tables of n_cal calibrations (aiy_panel_build): m_pol/c_pol
    [n_cal, S, n_M, n_a + 1] device tensors -> uint8 tensor [n_cal, table bytes]
    (unemployed: with the unemployed sub-states' cells, Krusell-Smith mode)."""
    n_cal, S, n_M, n1 = m_pol.shape
    nbytes = int(h.lib.aiy_panel_table_bytes(n_lab, n_M, n1 - 1, int(bool(unemployed))))
    if nbytes <= 0:
        raise _lib.AiyagariLibError(f"unsupported panel table sizes n_lab={n_lab} n_M={n_M} n_a={n1 - 1}")
    tables = torch.empty((n_cal, nbytes), dtype=torch.uint8, device=device)
    m_pol = m_pol.contiguous()
    c_pol = c_pol.contiguous()
    h.check(h.lib.aiy_panel_build(h.h, n_cal, S, n_M, n1 - 1, n_lab, int(bool(unemployed)), _lib.ptr(m_pol),
                                  _lib.ptr(c_pol), _lib.ptr(tables), _lib.stream_ptr()), "aiy_panel_build")
    return tables


def run_block(h, pb, markets_ref, n_agents, a, lab, seeds, ge_iter, t0, n_periods, act_T, sow, hist_A, hist_M,
              shock_mode, u_host_source, chunk, sp, stream, emp_source=None):
    """aiy_sim_block_periods over [t0, t0 + n_periods): Philox in one call, host uniforms
    (u_host_source(n) -> [n_cal][n][n_agents] or, for one calibration, [n][n_agents]) and
    employment states (emp_source, same shapes) in chunks of ``chunk`` periods."""
    if shock_mode == "philox" and emp_source is None:
        h.check(h.lib.aiy_sim_block_periods(h.h, ctypes.byref(pb), markets_ref, n_agents, _lib.ptr(a), _lib.ptr(lab),
                                            None, None, seeds, int(ge_iter), int(t0), int(n_periods), int(act_T),
                                            _lib.ptr(sow), _lib.ptr(hist_A), _lib.ptr(hist_M), sp),
                "aiy_sim_block_periods")
        return
    if shock_mode not in ("philox", "numpy"):
        raise ValueError(shock_mode)

    def block(source, n, dtype):
        x = np.ascontiguousarray(source(n), dtype=dtype)
        want = (pb.n_cal, n, n_agents)
        if x.shape != want and not (pb.n_cal == 1 and x.shape == want[1:]):
            raise ValueError(f"host block shape {x.shape} != {want}")
        return torch.from_numpy(x.reshape(want)).to(a.device)

    t, end = t0, t0 + n_periods
    while t < end:
        n = min(chunk, end - t)
        ud = block(u_host_source, n, np.float64) if shock_mode == "numpy" else None
        ed = block(emp_source, n, np.uint8) if emp_source is not None else None
        h.check(h.lib.aiy_sim_block_periods(h.h, ctypes.byref(pb), markets_ref, n_agents, _lib.ptr(a), _lib.ptr(lab),
                                            _lib.ptr(ud), _lib.ptr(ed), seeds, int(ge_iter), int(t), int(n),
                                            int(act_T), _lib.ptr(sow), _lib.ptr(hist_A), _lib.ptr(hist_M), sp),
                "aiy_sim_block_periods")
        torch.cuda.current_stream(a.device).synchronize() if stream is None else stream.synchronize()
        del ud, ed
        t += n


class BatchedPanel:
    """Panels of n_cal independent calibrations (same S, n_M, n_a, n_lab and population
    size), simulated together by the block engine: one launch covers every
    calibration's periods.  Tensors are stacked over calibrations."""

    def __init__(self, n_cal: int, n_agents: int, act_T: int, device=None):
        self.device = torch.device(device or "cuda")
        self.n_cal, self.n_agents, self.act_T = int(n_cal), int(n_agents), int(act_T)
        self.a = torch.empty((n_cal, n_agents), dtype=F64, device=self.device)
        self.lab = torch.empty((n_cal, n_agents), dtype=torch.uint8, device=self.device)
        self.sow = torch.zeros((n_cal, _lib.AIY_SOW_DOUBLES), dtype=F64, device=self.device)
        self.hist_A = torch.zeros((n_cal, act_T), dtype=F64, device=self.device)
        self.hist_M = torch.zeros((n_cal, act_T), dtype=F64, device=self.device)
        self._model = None

    def reset(self, a0, lab0, sow0):
        """a0 [n_cal] or [n_cal, n_agents]; lab0 [n_cal, n_agents]; sow0 [n_cal, 5]
        (Mnow, Aprev, Mrkv, Rnow, Wnow)."""
        a0 = np.asarray(a0, dtype=np.float64)
        a0 = np.broadcast_to(a0[:, None] if a0.ndim == 1 else a0, (self.n_cal, self.n_agents))
        self.a.copy_(torch.from_numpy(np.array(a0, dtype=np.float64, order="C")))
        self.lab.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(lab0, dtype=np.uint8))))
        sow = np.zeros((self.n_cal, _lib.AIY_SOW_DOUBLES))
        sow[:, :5] = np.asarray(sow0, dtype=np.float64)
        self.sow.copy_(torch.from_numpy(sow))
        self.hist_A.zero_()
        self.hist_M.zero_()

    def bind_models(self, m_pol, c_pol, M_grid, lab_level, lab_cdf, mrkv_hist, markets):
        """m_pol/c_pol [n_cal, S, n_M, n1] device; M_grid [n_cal, n_M]; lab_level
        [n_cal, n_lab]; lab_cdf [n_cal, n_lab, n_lab]; mrkv_hist [n_cal, act_T];
        markets: list of n_cal dicts (see make_market)."""
        n_cal, S, n_M, n1 = m_pol.shape
        if n_cal != self.n_cal:
            raise ValueError("calibration count mismatch")
        n_lab = int(lab_level.shape[1])
        h = _lib.handle(self.device.index)
        keep = dict(M_grid=M_grid.contiguous(), lab_level=lab_level.contiguous(), lab_cdf=lab_cdf.contiguous(),
                    mrkv_hist=mrkv_hist.to(torch.int32).contiguous())
        keep["tables"] = build_tables(h, m_pol, c_pol, n_lab, self.device)
        pb = _lib.PanelBatch(n_cal, S, n_M, n1 - 1, n_lab, *(_lib.ptr(keep[k]) for k in
                                                              ("tables", "M_grid", "lab_level", "lab_cdf",
                                                               "mrkv_hist")), 0)
        mks = (_lib.Market * n_cal)(*(make_market(m) for m in markets))
        self._model = (pb, mks, keep)

    def run(self, t0, n_periods, shock_mode="philox", seeds=None, ge_iter=0, u_host_source=None, chunk=1000,
            stream=None):
        if self._model is None:
            raise RuntimeError("bind_models() first")
        pb, mks, _ = self._model
        h = _lib.handle(self.device.index)
        seeds = [0] * self.n_cal if seeds is None else list(seeds)
        sd = (ctypes.c_uint64 * self.n_cal)(*(int(x) & ((1 << 64) - 1) for x in seeds))
        run_block(h, pb, mks, self.n_agents, self.a, self.lab, sd, ge_iter, t0, n_periods, self.act_T, self.sow,
                  self.hist_A, self.hist_M, shock_mode, u_host_source, chunk, _lib.stream_ptr(stream), stream)
